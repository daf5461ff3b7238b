"""A/B of svo_render_progressive_async's readback: per-frame host time of
the C3 1080p progressive loop through the pipelined entry point, with the frame's RGBA8 words
moved to the pinned slot by one DMA copy (svo_config.readback 0), a kernel writing the mapped pinned
buffer (1) or two DMA copies on two streams (2), and one DMA copy of 3-byte pixels (RGB24); the
blocking svo_render_progressive beside.
Every mode's displayed frames are compared with the blocking path's for the same samples.
Also times a plain pinned D2H of the same 8.3 MB (torch) for the link's rate.

  python tools/readback_ab.py [--frames 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    a = ap.parse_args()
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = CONFIGS["C3"]
    W, H = cfg["width"], cfg["height"]
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"], device=0)
    cam = CAMERAS["flyover"]()
    out = {"frame": f"{W}x{H}", "frames": a.frames}

    src = torch.empty(W * H, dtype=torch.int32, device="cuda")
    dst = torch.empty(W * H, dtype=torch.int32).pin_memory()
    for _ in range(5):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(50):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) / 50 * 1e3
    out["pinned_d2h_8.3MB"] = {"ms": round(ms, 4), "GB_per_s": round(W * H * 4 / (ms * 1e-3) / 1e9, 1)}

    ref = []
    with RaytracingMaster(device=0, capacity_nodes=len(svo)) as rm:
        rm.SetSVOBuffer(svo)
        rm.UpdateShaderParameters(cam, W, H)
        for _ in range(3):
            rm.RenderProgressive(W, H)
        rm.currentSample = 0
        t = time.perf_counter()
        for _ in range(20):
            f, _ = rm.RenderProgressive(W, H)
            ref.append(f.copy())
        out["blocking_svo_render_progressive_ms"] = round((time.perf_counter() - t) / 20 * 1e3, 4)
    for mode, rgb in ((0, False), (1, False), (2, False), (0, True)):
        key = f"async_push{mode}" + ("_rgb24" if rgb else "")
        with RaytracingMaster(device=0, capacity_nodes=len(svo), config={"readback": mode}) as rm:
            rm.SetSVOBuffer(svo)
            rm.UpdateShaderParameters(cam, W, H)
            got = []
            for i in range(21):   # the same 20 samples as the blocking run (+1 call to get the 20th back)
                f = rm.RenderProgressiveAsync(W, H, rgb=rgb)
                if f is not None:
                    if rgb:   # back to display words for the comparison
                        f = f.astype(np.uint32)
                        f = f[..., 0] | (f[..., 1] << 8) | (f[..., 2] << 16) | np.uint32(255 << 24)
                    got.append(f)
            bad = sum(int(not np.array_equal(g, r)) for g, r in zip(got, ref))
            rm.currentSample = 0
            for _ in range(10):
                rm.RenderProgressiveAsync(W, H, copy=False, rgb=rgb)
            t = time.perf_counter()
            for _ in range(a.frames):
                rm.RenderProgressiveAsync(W, H, copy=False, rgb=rgb)
            ms = (time.perf_counter() - t) / a.frames * 1e3
        out[key] = {"ms_per_frame": round(ms, 4), "frames_compared": len(got), "frames_differing_from_blocking": bad,
                    "bytes_per_frame": W * H * (3 if rgb else 4)}
        print(json.dumps({key: out[key]}), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
