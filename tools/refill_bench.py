"""Experiment: the lane-refill kernel (env SVO_REFILL=K,T[,paired]; VERDICT r1
item 9) against the default tile kernel on the C3 flyover frame (and the Main
pose), one MI355X.  Kernel time = the library's HIP events around the
primary-ray kernel alone (svo_set_options(SVO_OPT_KERNEL_TIMING)), mean of
--steps launches after warmup; every variant's hit records are compared with the
default kernel's.

  python tools/refill_bench.py [--steps 40] [--configs 2,16 4,16 4,32 8,32 4,16,1]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--configs", nargs="+", default=["2,8", "2,16", "4,16", "4,32", "8,32", "2,16,1", "4,16,1"])
    ap.add_argument("--cameras", nargs="+", default=["flyover", "main"])
    a = ap.parse_args()
    import torch
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    svo = build_sampler_svo(4, 11, device=0)
    W, H = 1920, 1080
    s = torch.cuda.Stream()
    hits = torch.empty(W * H * 24, dtype=torch.uint8, device="cuda")
    rgba = torch.empty(W * H * 4, dtype=torch.float32, device="cuda")

    def run(cam, env):
        for k in ("SVO_REFILL", "SVO_XCD_REMAP"):
            os.environ.pop(k, None)
        os.environ.update(env)
        rm = RaytracingMaster(device=0, capacity_nodes=len(svo))   # SVO_XCD_REMAP is read here
        rm.SetSVOBuffer(svo)
        rm.UpdateShaderParameters(CAMERAS[cam](), W, H)
        for _ in range(8):
            rm.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), stream=s.cuda_stream)
        s.synchronize()
        rm.set_kernel_timing(True)
        rm.kernel_time()
        for _ in range(a.steps):
            rm.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), stream=s.cuda_stream)
        s.synchronize()
        ms, n = rm.kernel_time()
        rm.close()
        return ms, hits.clone()

    for cam in a.cameras:
        base, ref = run(cam, {})
        base0, _ = run(cam, {"SVO_XCD_REMAP": "0"})
        print(f"{cam}: tile kernel {base:.4f} ms (XCD strips, default), {base0:.4f} ms (raster tile order)",
              flush=True)
        for c in a.configs:
            env = {"SVO_REFILL": c}
            if c.count(",") == 2:
                env["SVO_XCD_REMAP"] = "0"
            ms, h = run(cam, env)
            same = bool(torch.equal(h, ref))
            k, t = c.split(",")[:2]
            kind = "cost-paired lists" if c.count(",") == 2 else "neighbouring tiles"
            print(f"  refill K={k} T={t} ({kind}): {ms:.4f} ms = {ms / base:.3f}x the tile kernel; "
                  f"hit records identical: {same}", flush=True)


if __name__ == "__main__":
    main()
