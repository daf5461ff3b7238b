"""A/B of the render loop's latency form (trace_lat, svo_config.loop_form 1) against the lean loop
(loop_form 0) and the library's automatic choice (loop_form -1) on launches of decreasing size: the whole C3 frame, one rank's band of the strong
1920x1080 split at N = 2, 4, 8 (round-robin 8-row bands), and the tile row holding the
frame's heaviest tile alone.  Kernel time = the library's HIP events around the render
kernel (mean of K launches after warmup).  Both contexts render the same frame; their hit
records must be identical (the forms make the same decisions).

  python tools/lat_ab.py [--config C3] [--camera flyover] [--reps 30]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--camera", default=None)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--heavy-row", type=int, default=80, help="tile row of the heaviest tile (wave_log --tile-row -2)")
    a = ap.parse_args()
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster, band_rows
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = CONFIGS[a.config]
    W, H, mode = cfg["width"], cfg["height"], cfg["stack_mode"]
    cam = CAMERAS[a.camera or cfg["camera"]]()
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    ctx = {}
    for name, lat in (("lean", 0), ("lat", 1), ("auto", -1)):
        rm = RaytracingMaster(capacity_nodes=len(svo), config={"loop_form": lat})
        rm.SetSVOBuffer(svo)
        rm.UpdateShaderParameters(cam, W, H)
        ctx[name] = rm
    cases = [("frame", None), ("band N=2", (8, 1, 2)), ("band N=4", (8, 1, 4)), ("band N=8", (8, 1, 8)),
             (f"tile row {a.heavy_row}", (8, a.heavy_row, (H + 7) // 8))]
    s = torch.cuda.Stream()
    for label, band in cases:
        rows = H if band is None else len(band_rows(H, band))
        out = {}
        hits = {}
        for name, rm in ctx.items():
            h = torch.empty(rows * W * 24, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            for _ in range(5):
                rm.render_device(W, H, hits_ptr=h.data_ptr(), band=band, stack_mode=mode, stream=s.cuda_stream)
            torch.cuda.synchronize()
            rm.set_kernel_timing(True)
            rm.kernel_time()
            for _ in range(a.reps):
                rm.render_device(W, H, hits_ptr=h.data_ptr(), band=band, stack_mode=mode, stream=s.cuda_stream)
            ms, n = rm.kernel_time()
            rm.set_kernel_timing(False)
            torch.cuda.synchronize()
            out[name] = ms
            hits[name] = h.cpu().numpy()
        same = np.array_equal(hits["lean"], hits["lat"]) and np.array_equal(hits["lean"], hits["auto"])
        tiles = ((W + 7) // 8) * ((rows + 7) // 8)
        print(f"{label:>14}: {tiles:6d} tiles  lean {out['lean'] * 1e3:8.1f} us  lat {out['lat'] * 1e3:8.1f} us  "
              f"lat/lean {out['lat'] / out['lean']:.3f}  auto {out['auto'] * 1e3:8.1f} us  "
              f"hit records identical: {same}", flush=True)
        if not same:
            raise SystemExit("latency form and lean loop disagree")
    for rm in ctx.values():
        rm.close()


if __name__ == "__main__":
    main()
