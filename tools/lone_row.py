"""Render one tile row of a config's frame alone (or the whole frame), K times, for PMC passes
on the lone-wave case (tools/pmc_lone_row.sh): the row holding the frame's heaviest tile runs
one wave per CU, so its time is the heaviest wave's own chain.

  python tools/lone_row.py [--config C3] [--row 80 | --row -1 (whole frame)] [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--camera", default=None)
    ap.add_argument("--row", type=int, default=80)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster, band_rows
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = CONFIGS[a.config]
    W, H, mode = cfg["width"], cfg["height"], cfg["stack_mode"]
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    rm = RaytracingMaster(capacity_nodes=len(svo))
    rm.SetSVOBuffer(svo)
    rm.UpdateShaderParameters(CAMERAS[a.camera or cfg["camera"]](), W, H)
    band = None if a.row < 0 else (8, a.row, (H + 7) // 8)
    rows = H if band is None else len(band_rows(H, band))
    h = torch.empty(rows * W * 24, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    for _ in range(5):
        rm.render_device(W, H, hits_ptr=h.data_ptr(), band=band, stack_mode=mode, stream=s.cuda_stream)
    torch.cuda.synchronize()
    rm.set_kernel_timing(True)
    rm.kernel_time()
    for _ in range(a.reps):
        rm.render_device(W, H, hits_ptr=h.data_ptr(), band=band, stack_mode=mode, stream=s.cuda_stream)
    ms, n = rm.kernel_time()
    torch.cuda.synchronize()
    print(f"{a.config} {'frame' if band is None else f'tile row {a.row}'}: {n} launches, kernel {ms * 1e3:.1f} us",
          flush=True)
    rm.close()


if __name__ == "__main__":
    main()
