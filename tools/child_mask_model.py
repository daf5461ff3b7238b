"""Model of a node format whose record carries its non-leaf children's valid / leaf masks
(VERDICT r3 item 3), on the heaviest C3 tiles, before building it.

Today (lean loop) a trip that follows a PUSH or a POP waits for the new node's fetch,
whatever the trip then does.  With the children's masks in the parent's record, a lane
that has just entered node P already holds P's masks (from the parent's record, or from
the stack entry on a POP), so its next iteration waits for a fetch only if it PUSHes again
(that needs P's own record: its `first` word and P's children's masks -- a load issued one
trip earlier, at the PUSH into P).  Per lane iteration i (oracle-checked iteration kinds,
tools/trip_kinds.py's float32 restatement of NVIDIASVO.compute:57-156):

  today      fetch-bound iff i == 0 or iteration i - 1 was PUSH / POP
  masks_pop  (masks kept on the stack) fetch-bound iff i == 0, or i - 1 was PUSH / POP and
             iteration i is a PUSH
  refetch    (8-byte stack, a POP re-fetches the ancestor's record) fetch-bound iff i == 0,
             i - 1 was a POP, or i - 1 was a PUSH and iteration i is a PUSH

A wave trip is fetch-bound if any active lane's iteration on it is.  The build criterion
(VERDICT r3 item 3): >= 10 % fewer fetch-bound wave trips on the heaviest tile.

  python tools/child_mask_model.py gpurun_out/c3_pool.npz [--camera flyover] [--tiles 16]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from trip_kinds import trace_kinds  # noqa: E402


def fetch_bound(ks):
    """(today, masks_pop, refetch) fetch-bound flags of one ray's iterations."""
    n = len(ks)
    today, mpop, refetch = np.zeros(n, bool), np.zeros(n, bool), np.zeros(n, bool)
    for i, k in enumerate(ks):
        prev = ks[i - 1] if i else None
        if i == 0:
            today[i] = mpop[i] = refetch[i] = True
            continue
        entered = prev in ("PUSH", "POP")
        today[i] = entered
        mpop[i] = entered and k == "PUSH"
        refetch[i] = prev == "POP" or (prev == "PUSH" and k == "PUSH")
    return today, mpop, refetch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--camera", default="flyover")
    ap.add_argument("--tiles", type=int, default=16)
    a = ap.parse_args()
    from oracle import oracle as orc
    from raytracingtest_amd.camera import CAMERAS, main_light
    W, H = 1920, 1080
    z = np.load(a.npz)
    nodes = z["nodes"]
    svo = orc.OracleSVO(nodes=nodes, attachments=z["attachments"])
    c2w, inv_proj = CAMERAS[a.camera]().uniforms(W, H)
    cam = orc.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
    _, _, iters = orc.render(svo, cam, W, H, orc.STACK_HLSL | orc.COUNT_ITERS, want_rgba=False)
    it = iters.reshape(H, W).astype(np.int64)
    tx, ty = W // 8, H // 8
    tiles = it[:ty * 8, :tx * 8].reshape(ty, 8, tx, 8).transpose(0, 2, 1, 3).reshape(ty * tx, 64)
    cost = tiles.max(1)
    order = np.argsort(-cost)[:a.tiles]
    nodes_l = nodes.tolist()
    tot = np.zeros(4, np.int64)
    print(f"{'tile':>7} {'wave trips':>10} {'today':>7} {'masks_pop':>10} {'refetch':>8}   (fetch-bound wave trips)")
    for k in order:
        r0, c0 = divmod(int(k), tx)
        n = int(cost[k])
        wt = np.zeros((3, n), bool)
        for j in range(64):
            y, x = r0 * 8 + j // 8, c0 * 8 + j % 8
            o, d = orc.camera_ray(cam, x, y, W, H)
            ks = trace_kinds(nodes_l, o, d)
            if len(ks) != it[y, x]:
                raise SystemExit(f"restatement disagrees with the oracle at ({x}, {y}): {len(ks)} vs {it[y, x]}")
            for f, flags in enumerate(fetch_bound(ks)):
                wt[f, :len(flags)] |= flags
        c = wt.sum(1)
        tot += [n, *c]
        print(f"{int(k):7d} {n:10d} {c[0]:7d} {c[1]:6d} ({100.0 * (1 - c[1] / c[0]):4.1f}% fewer) "
              f"{c[2]:5d} ({100.0 * (1 - c[2] / c[0]):4.1f}% fewer)", flush=True)
    print(f"all {a.tiles} tiles: wave trips {tot[0]}, fetch-bound today {tot[1]} ({100.0 * tot[1] / tot[0]:.1f} %), "
          f"masks_pop {tot[2]} ({100.0 * (1 - tot[2] / tot[1]):.1f} % fewer), "
          f"refetch {tot[3]} ({100.0 * (1 - tot[3] / tot[1]):.1f} % fewer)")


if __name__ == "__main__":
    main()
