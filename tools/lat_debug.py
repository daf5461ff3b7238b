"""The automatic loop-form choice across camera jumps, submitted the way bench.py's
extra_poses does (10 + 20 launches per pose, no host sync between them): prints the
library's decisions (SVO_DEBUG=1: one 'svo lat:' line per order build) and each pose's kernel time.  A pose must get the
form its own costs call for, not the previous pose's.

  python tools/lat_debug.py [--config C3]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["SVO_DEBUG"] = "1"   # read when a context is created


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    a = ap.parse_args()
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = CONFIGS[a.config]
    W, H, mode = cfg["width"], cfg["height"], cfg["stack_mode"]
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    rm = RaytracingMaster(capacity_nodes=len(svo))
    rm.SetSVOBuffer(svo)
    h = torch.empty(W * H * 24, dtype=torch.uint8, device="cuda")
    rg = torch.empty(W * H * 4, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    for pose in ("flyover", "overview", "main", "terrain", "overview", "flyover"):
        rm.UpdateShaderParameters(CAMERAS[pose](), W, H)
        print(f"== pose {pose}", file=sys.stderr, flush=True)
        for _ in range(10):
            rm.render_device(W, H, hits_ptr=h.data_ptr(), rgba_ptr=rg.data_ptr(), stack_mode=mode, stream=s.cuda_stream)
        rm.set_kernel_timing(True)
        rm.kernel_time()
        for _ in range(20):
            rm.render_device(W, H, hits_ptr=h.data_ptr(), rgba_ptr=rg.data_ptr(), stack_mode=mode, stream=s.cuda_stream)
        ms, _ = rm.kernel_time()
        rm.set_kernel_timing(False)
        torch.cuda.synchronize()
        print(f"   {pose}: kernel {ms * 1e3:.1f} us", file=sys.stderr, flush=True)
    # a moving camera: a new view every launch (the interactive case), submitted without host
    # syncs; the decisions must keep arriving (a few frames late) instead of freezing
    from raytracingtest_amd.camera import OVERVIEW_EYE, OVERVIEW_TARGET, overview_camera
    print("== moving camera: overview eye orbiting, 120 launches, one view each", file=sys.stderr, flush=True)
    rm.set_kernel_timing(True)
    rm.kernel_time()
    for i in range(120):
        a_ = 0.01 * i
        eye = (OVERVIEW_EYE[0] + 5.0 * np.sin(a_), OVERVIEW_EYE[1], OVERVIEW_EYE[2] + 5.0 * (1.0 - np.cos(a_)))
        rm.UpdateShaderParameters(overview_camera(eye, OVERVIEW_TARGET), W, H)
        rm.render_device(W, H, hits_ptr=h.data_ptr(), rgba_ptr=rg.data_ptr(), stack_mode=mode, stream=s.cuda_stream)
    t = rm.stage_times()
    rm.set_kernel_timing(False)
    print(f"   moving: kernel mean {np.mean(t) * 1e3:.1f} us, first 10 {np.mean(t[:10]) * 1e3:.1f} us, "
          f"last 60 {np.mean(t[60:]) * 1e3:.1f} us", file=sys.stderr, flush=True)
    rm.close()


if __name__ == "__main__":
    main()
