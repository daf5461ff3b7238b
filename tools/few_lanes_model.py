"""How many wave trips of a frame run with few active lanes (oracle per-ray iteration
counts, lean loop: a lane is active for exactly its ray's iteration count).  The
question behind it: would a cheaper loop for waves with <= k active lanes (uniform
branches instead of the lane-mask form of every path) shorten the heaviest waves?
Only if their last trips run with few lanes -- this prints that, per camera.

  python tools/few_lanes_model.py gpurun_out/r03n/c3_pool.npz
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
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    from oracle import oracle as orc
    from raytracingtest_amd.camera import CAMERAS, main_light
    z = np.load(a.npz)
    svo = orc.OracleSVO(nodes=z["nodes"], attachments=z["attachments"])
    W, H = 1920, 1080
    for name in ("flyover", "overview", "main", "terrain"):
        c2w, inv_proj = CAMERAS[name]().uniforms(W, H)
        cam = orc.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
        _, _, iters = orc.render(svo, cam, W, H, orc.STACK_HLSL | orc.COUNT_ITERS, want_rgba=False)
        it = iters.reshape(H, W).astype(np.int64)
        tx, ty = W // 8, H // 8
        tiles = it[:ty * 8, :tx * 8].reshape(ty, 8, tx, 8).transpose(0, 2, 1, 3).reshape(ty * tx, 64)
        s = np.sort(tiles, axis=1)[:, ::-1]
        mx = s[:, 0]
        tot = int(mx.sum())
        print(f"== {name}: wave trips {tot}, heaviest tile {int(mx.max())}")
        for k in (1, 2, 4, 8):
            few = int((mx - s[:, k]).sum())
            print(f"   trips with <= {k} active lanes: {few} ({100.0 * few / tot:.1f} %)")
        for t in np.argsort(-mx)[:a.top]:
            print(f"   tile {int(t):6d}: lane iterations, heaviest first: {s[t, 0]}, {s[t, 1]}, {s[t, 2]}, "
                  f"5th {s[t, 4]}, 9th {s[t, 8]}  (trips with <= 2 lanes: {s[t, 0] - s[t, 2]})")


if __name__ == "__main__":
    main()
