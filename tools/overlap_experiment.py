"""Experiment: does overlapping consecutive frames (launches on S streams, each
with its own output buffers) raise single-GPU throughput?  The render kernel's
frame time is close to its heaviest wave's latency, so the
ramp-down tail leaves SIMDs idle; a second frame in flight could fill them.

Usage (GPU): python tools/overlap_experiment.py [--streams 1 2 3] [--steps 60]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--camera", default="flyover")
    ap.add_argument("--separate", action="store_true",
                    help="one context (own pool copy) per stream instead of one shared context")
    a = ap.parse_args()
    import torch
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    svo = build_sampler_svo(4, 11, device=0)
    W, H = 1920, 1080
    for S in a.streams:
        # one context: the plugin keeps per-stream dispatch-order state, so its renders on
        # different streams overlap over one pool; --separate: a context (pool copy) per stream
        n_ctx = S if a.separate else 1
        rms = [RaytracingMaster(device=0, capacity_nodes=len(svo)) for _ in range(n_ctx)]
        for rm in rms:
            rm.SetSVOBuffer(svo)
            rm.UpdateShaderParameters(CAMERAS[a.camera](), W, H)
        streams = [torch.cuda.Stream() for _ in range(S)]
        hits = [torch.empty(W * H * 24, dtype=torch.uint8, device="cuda") for _ in range(S)]
        rgba = [torch.empty(W * H * 4, dtype=torch.float32, device="cuda") for _ in range(S)]

        def step(i):
            k = i % S
            rms[k % n_ctx].render_device(W, H, rgba_ptr=rgba[k].data_ptr(), hits_ptr=hits[k].data_ptr(),
                             stream=streams[k].cuda_stream)

        for i in range(10):
            step(i)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(a.steps):
            step(i)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / a.steps * 1e3
        print(f"streams={S}: {ms:.4f} ms/frame, {W * H / ms / 1e3:.1f} Mrays/s", flush=True)
        for rm in rms:
            rm.close()


if __name__ == "__main__":
    main()
