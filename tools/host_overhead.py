"""Experiment: host time per call of the N > 1 step's plugin calls (bench.py Gather:
render_frame with a weighted-deal band, assemble_frame of N-1 parts), issued
back to back on a tiny frame so the GPU never holds the host back.  At N = 8 a
C3 step gives the host ~120 us to issue everything (render, gather, assemble)
before the GPU idles.

  python tools/host_overhead.py [--calls 2000] [--world 8]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--world", type=int, default=8)
    a = ap.parse_args()
    import torch
    from raytracingtest_amd import RaytracingMaster, _lib
    from raytracingtest_amd import distributed as D
    from raytracingtest_amd.builder import build_menger
    from raytracingtest_amd.camera import overview_camera
    svo = build_menger(5)
    W, H = 64, 64 * a.world
    rm = RaytracingMaster(device=0, capacity_nodes=len(svo))
    rm.SetSVOBuffer(svo)
    rm.UpdateShaderParameters(overview_camera(), W, H)
    s = torch.cuda.Stream()
    owner = D.weighted_owner(a.world, 0.75)
    band = D.rank_band(1, a.world, owner=owner)
    n = D.max_band_len(H, a.world, owner=owner) * W
    buf = torch.empty(n * 3, dtype=torch.uint8, device="cuda")
    frame = torch.empty(W * H, dtype=torch.int32, device="cuda")
    parts = [None] + [torch.zeros(n * 3, dtype=torch.uint8, device="cuda") for _ in range(1, a.world)]
    ptrs = [None] + [p.data_ptr() for p in parts[1:]]

    def timed(fn):
        for _ in range(50):
            fn()
        s.synchronize()
        t = time.perf_counter()
        for _ in range(a.calls):
            fn()
        host = (time.perf_counter() - t) / a.calls * 1e6
        s.synchronize()
        return host

    r = timed(lambda: rm.render_frame(W, H, rgb8=buf.data_ptr(), band=band, stream=s.cuda_stream))
    asm = timed(lambda: rm.assemble_frame(W, H, ptrs, _lib.PART_RGB8, rgba8=frame.data_ptr(), skip_part=0,
                                          stream=s.cuda_stream, owner=owner))
    import ctypes
    band_c = _lib.make_band(band)
    deal_c = _lib.make_band((8, 0, a.world, tuple(owner)))
    parts_c = (ctypes.c_void_p * a.world)(*ptrs)
    rc = timed(lambda: rm.render_frame(W, H, rgb8=buf.data_ptr(), band=band_c, stream=s.cuda_stream))
    asmc = timed(lambda: rm.assemble_frame(W, H, parts_c, _lib.PART_RGB8, rgba8=frame.data_ptr(), skip_part=0,
                                           stream=s.cuda_stream, deal=deal_c))
    ev = torch.cuda.Event()
    e = timed(lambda: (ev.record(s), s.wait_event(ev)))
    print(f"host us per call (world {a.world}, weighted deal of {len(owner)} bands): render_frame {r:.1f}, "
          f"assemble_frame {asm:.1f}, event record + wait {e:.1f}; with the band / deal / parts structs built "
          f"once (bench.py Gather): render_frame {rc:.1f}, assemble_frame {asmc:.1f}", flush=True)


if __name__ == "__main__":
    main()
