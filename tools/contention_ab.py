"""What slows the heaviest wave inside a full frame (~1,016 cycles per trip in the
frame against ~835 alone)?  The C3 frame's heaviest tile row (240 waves, one per CU, lean loop)
renders while tools/filler.hip occupies ~7 of every SIMD's 8 wave slots with one kind of load:
no filler, VALU only, L1-resident gathers, L2-resident gathers.  The row's kernel time under each
says whether the heavy wave loses its time to issue contention on its SIMD or to the memory path.

  hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/build/libfiller.so tools/filler.hip
  python tools/contention_ab.py [--reps 20]
"""
import argparse
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--row", type=int, default=80)
    ap.add_argument("--waves", type=int, default=7 * 1024)
    a = ap.parse_args()
    os.environ["SVO_LAT"] = "0"
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "build", "libfiller.so"))
    lib.filler_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_ulonglong, ctypes.c_void_p, ctypes.c_uint,
                                  ctypes.c_void_p, ctypes.c_void_p]
    cfg = CONFIGS["C3"]
    W, H = cfg["width"], cfg["height"]
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    rm = RaytracingMaster(capacity_nodes=len(svo))
    rm.SetSVOBuffer(svo)
    rm.UpdateShaderParameters(CAMERAS["flyover"](), W, H)
    g = torch.Generator().manual_seed(3)
    tables = {2: (torch.randint(0, 2048, (2048, 2), generator=g, dtype=torch.int32).cuda(), 2047),
              3: (torch.randint(0, 1 << 18, (1 << 18, 2), generator=g, dtype=torch.int32).cuda(), (1 << 18) - 1)}
    sink = torch.zeros(a.waves, dtype=torch.float32, device="cuda")
    # separate hardware queues: with GPU_MAX_HW_QUEUES = 4, two ordinary streams may share one and
    # serialise; a high-priority stream for the row takes a queue of its own
    sf, sr = torch.cuda.Stream(), torch.cuda.Stream(priority=-1)
    band = (8, a.row, (H + 7) // 8)
    h = torch.empty(8 * W * 24, dtype=torch.uint8, device="cuda")
    hf = torch.empty(H * W * 24, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for _ in range(300):   # the clock ramp: reach the sustained clock first
        rm.render_device(W, H, hits_ptr=hf.data_ptr(), stack_mode=0, stream=sr.cuda_stream)
    for _ in range(10):
        rm.render_device(W, H, hits_ptr=h.data_ptr(), band=band, stack_mode=0, stream=sr.cuda_stream)
    torch.cuda.synchronize()
    names = {0: "no filler", 1: "VALU filler", 2: "L1-gather filler", 3: "L2-gather filler"}
    for rnd in range(2):
        for mode in (0, 1, 2, 3):
            rm.set_kernel_timing(True)
            rm.kernel_time()
            for _ in range(a.reps):
                if mode:
                    t, m = tables.get(mode, tables[2])
                    rc = lib.filler_launch(mode, a.waves, 40000, t.data_ptr(), m, sink.data_ptr(), sf.cuda_stream)
                    if rc:
                        raise SystemExit(f"filler launch failed: {rc}")
                    time.sleep(50e-6)   # let the filler's waves become resident first
                rm.render_device(W, H, hits_ptr=h.data_ptr(), band=band, stack_mode=0, stream=sr.cuda_stream)
                torch.cuda.synchronize()
            ms, n = rm.kernel_time()
            rm.set_kernel_timing(False)
            print(f"round {rnd}  filler waves {a.waves}  {names[mode]:18s} tile row {a.row}: {n} launches, kernel {ms * 1e3:6.1f} us", flush=True)
    rm.close()


if __name__ == "__main__":
    main()
