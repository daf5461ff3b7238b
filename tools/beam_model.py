"""Upper bound of a per-tile "beam" start (Laine & Karras 2010, sec. 5: trace a coarse beam
per 8x8 tile first, then start every ray of the tile at the beam's conservative distance):
with the oracle on the C3 pool (tools/dump_pool.py), the per-tile wave trips (max over the
tile's 64 rays) when every ray restarts at the tile's *first hit distance* (the perfect
beam: min over the tile's hit rays, times 1 - eps), against the full traversal.  A real beam
can only be worse.  Only the heaviest tiles are re-traced (they bound the launch).

  python tools/beam_model.py gpurun_out/r03b/c3_pool.npz [--camera flyover] [--top 512]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--camera", default="flyover")
    ap.add_argument("--top", type=int, default=512)
    ap.add_argument("--eps", type=float, default=1e-3)
    a = ap.parse_args()
    from oracle import oracle as orc
    from raytracingtest_amd.camera import CAMERAS, main_light
    W, H = 1920, 1080
    z = np.load(a.npz)
    svo = orc.OracleSVO(nodes=z["nodes"], attachments=z["attachments"])
    c2w, inv_proj = CAMERAS[a.camera]().uniforms(W, H)
    cam = orc.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
    hits, _, iters = orc.render(svo, cam, W, H, orc.STACK_HLSL | orc.COUNT_ITERS, want_rgba=False)
    it = iters.reshape(H, W).astype(np.int64)
    th = hits["t"].reshape(H, W)
    tx, ty = W // 8, H // 8
    tiles = it[:ty * 8, :tx * 8].reshape(ty, 8, tx, 8).transpose(0, 2, 1, 3).reshape(ty * tx, 64)
    tt = th[:ty * 8, :tx * 8].reshape(ty, 8, tx, 8).transpose(0, 2, 1, 3).reshape(ty * tx, 64)
    cost = tiles.max(1)
    order = np.argsort(-cost)[:a.top]
    new_cost = cost.copy()
    for k in order:
        t_beam = np.min(tt[k])
        if not np.isfinite(t_beam):
            continue
        t_beam *= 1.0 - a.eps
        r0, c0 = divmod(int(k), tx)
        m = 0
        for j in range(64):
            y, x = r0 * 8 + j // 8, c0 * 8 + j % 8
            o, d = orc.camera_ray(cam, x, y, W, H)
            o2 = (o + np.float32(t_beam / 64.0) * d).astype(np.float32)   # hit t = 2048 x cube t; world = 32 x cube
            _, _, _, n = orc.intersect(svo, o2, d)
            m = max(m, n)
        new_cost[k] = m
    top = cost[order]
    top_new = new_cost[order]
    print(f"{a.camera}: {len(cost)} tiles, total wave trips {cost.sum()} -> {new_cost.sum()} "
          f"(only the top {a.top} re-traced)")
    for q in (1, 8, 64, 256, a.top):
        q = min(q, a.top)
        print(f"  top-{q:<4d} tiles: max {top[:q].max():4d} -> {top_new[:q].max():4d}   "
              f"mean {top[:q].mean():7.1f} -> {top_new[:q].mean():7.1f}")
    print(f"  heaviest tile after the beam start: {new_cost.max()} (was {cost.max()})")


if __name__ == "__main__":
    main()
