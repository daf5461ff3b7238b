"""SIMD efficiency of 8x8-tile primary-ray traversal (diagnostics).

Builds the bench SVO on cuda:0, traces the frame with the CPU oracle counting
loop iterations per ray, and reports, per 8x8 tile (one wave64 of the tile
kernel): sum of ray iterations vs 64 x the tile's max (the wave's trip count).
Optionally saves the SVO (--save) for CPU-side experiments.

  python tools/simd_efficiency.py [--camera flyover] [--max-level 11] [--save gpurun_out/c3_svo.npz]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--camera", default="flyover")
    ap.add_argument("--max-level", type=int, default=11)
    ap.add_argument("--save", default=None)
    ap.add_argument("--load", default=None, help="npz written by --save (no GPU needed)")
    ap.add_argument("--save-iters", default=None, help="npz of the per-ray iteration / fetch counts and hit flags")
    args = ap.parse_args()
    from oracle import oracle as orc
    from raytracingtest_amd.camera import CAMERAS, main_light

    if args.load:
        z = np.load(args.load)
        nodes, att = z["nodes"], z["attachments"]
    else:
        from raytracingtest_amd.native_builder import build_sampler_svo
        svo = build_sampler_svo(4, args.max_level, prefer_v1=False)
        nodes, att = svo.to_v2(), svo.attachments
        if args.save:
            np.savez_compressed(args.save, nodes=nodes, attachments=att)
    W, H = 1920, 1080
    cam = CAMERAS[args.camera]()
    c2w, inv_proj = cam.uniforms(W, H)
    ocam = orc.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
    osvo = orc.OracleSVO(nodes=nodes, attachments=att)
    hits, _, it = orc.render(osvo, ocam, W, H, orc.COUNT_ITERS, nthreads=min(16, os.cpu_count() or 1),
                             want_rgba=False)
    _, _, fe = orc.render(osvo, ocam, W, H, 0, nthreads=min(16, os.cpu_count() or 1), want_rgba=False)
    if args.save_iters:
        _, _, sit = orc.render(osvo, ocam, W, H, orc.SHADOW_RAYS | orc.COUNT_SHADOW_ITERS,
                               nthreads=min(16, os.cpu_count() or 1), want_rgba=False)
        np.savez_compressed(args.save_iters, iters=it.reshape(H, W).astype(np.uint16),
                            shadow_iters=sit.reshape(H, W).astype(np.uint16),
                            fetches=fe.reshape(H, W).astype(np.uint16),
                            hit=((hits["flags"] & 1) != 0).reshape(H, W))
    it = it.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64).astype(np.int64)
    fe = fe.reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64).astype(np.int64)
    hit = ((hits["flags"] & 1) != 0).reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
    tmax = it.max(1)
    print(f"rays {it.size}, iterations/ray {it.mean():.2f} (hit rays {it[hit].mean():.2f}, "
          f"miss {it[~hit].mean():.2f}), fetches/ray {fe.mean():.2f}")
    print(f"wave trips: sum {tmax.sum()}, mean {tmax.mean():.2f}, "
          f"SIMD efficiency {it.sum() / (64 * tmax.sum()):.3f}")
    q = np.percentile(tmax, [10, 50, 90, 99, 100])
    print("wave trips p10/p50/p90/p99/max", q)
    # lanes alive per trip, averaged over waves weighted by trips
    alive = np.zeros(int(tmax.max()) + 1)
    for k in range(1, len(alive)):
        alive[k] = (it >= k).sum()
    waves_at = np.array([(tmax >= k).sum() for k in range(len(alive))])
    print("mean active lanes per wave at trip k (k=1,5,10,20,40,80):",
          [round(alive[k] / max(waves_at[k], 1), 1) for k in (1, 5, 10, 20, 40, 80) if k < len(alive)])


if __name__ == "__main__":
    main()
