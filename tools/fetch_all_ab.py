"""A/B of the unpredicated node fetch (SVO_FETCH_ALL=1: every lane loads its node on every
trip) against the predicated one (SVO_FETCH_ALL=0: only lanes whose node changed) on a
config's whole frame at every camera pose.  The library picks by pool size (predicated
from 2^24 nodes, svo_rt.hip launch); this re-measures that rule on C4 / C5.  Kernel time =
the library's HIP events around the render kernel (mean of K launches); both contexts write
hit records + RGBA32F like bench.py's step, and their hit records must be identical.

  python tools/fetch_all_ab.py [--config C4] [--reps 20]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cameras", default="overview,terrain,main,flyover")
    a = ap.parse_args()
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = CONFIGS[a.config]
    W, H, mode = cfg["width"], cfg["height"], cfg["stack_mode"]
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    print(f"{a.config}: {len(svo)} nodes, {W}x{H}, stack mode {mode}", flush=True)
    ctx = {}
    for fa in ("0", "1"):
        os.environ["SVO_FETCH_ALL"] = fa
        rm = RaytracingMaster(capacity_nodes=len(svo))
        rm.SetSVOBuffer(svo)
        ctx[fa] = rm
    os.environ.pop("SVO_FETCH_ALL", None)
    hits = torch.empty(W * H * 24, dtype=torch.uint8, device="cuda")
    rgba = torch.empty(W * H * 16, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    for cam_name in a.cameras.split(","):
        cam = CAMERAS[cam_name]()
        times = {"0": [], "1": []}
        ref = None
        for rep in range(2):
            for fa, rm in ctx.items():
                rm.UpdateShaderParameters(cam, W, H)
                for _ in range(5):
                    rm.render_device(W, H, rgba_ptr=rgba.data_ptr(), hits_ptr=hits.data_ptr(), stack_mode=mode,
                                     stream=s.cuda_stream)
                torch.cuda.synchronize()
                rm.set_kernel_timing(True)
                rm.kernel_time()
                for _ in range(a.reps):
                    rm.render_device(W, H, rgba_ptr=rgba.data_ptr(), hits_ptr=hits.data_ptr(), stack_mode=mode,
                                     stream=s.cuda_stream)
                ms, _ = rm.kernel_time()
                rm.set_kernel_timing(False)
                torch.cuda.synchronize()
                times[fa].append(ms)
                h = hits.cpu().numpy()
                if ref is None:
                    ref = h
                elif not np.array_equal(ref, h):
                    raise SystemExit(f"{cam_name}: SVO_FETCH_ALL={fa} hit records differ")
        t0, t1 = (min(times[k]) for k in ("0", "1"))
        print(f"{cam_name:>9}: predicated {' / '.join(f'{t:.4f}' for t in times['0'])} ms  "
              f"unpredicated {' / '.join(f'{t:.4f}' for t in times['1'])} ms  "
              f"unpredicated/predicated {t1 / t0:.3f}  hit records identical", flush=True)
    for rm in ctx.values():
        rm.close()


if __name__ == "__main__":
    main()
