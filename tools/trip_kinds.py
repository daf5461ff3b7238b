"""What the heaviest tiles' loop trips do: a float32 Python restatement of the traversal loop
(oracle/svo_oracle.c orc_intersect_ex, HLSL stack mode, NVIDIASVO.compute:57-156) that labels
every iteration PUSH / HIT / ADVANCE (same node) / ADVANCE+POP, checked against the oracle's
own iteration count ray by ray.  Reports, for the heaviest tiles, the kinds' shares and the
wave trip count if every run of same-node ADVANCE iterations were folded into the trip that
follows it (an in-register sibling skip: no fetch, no stack traffic).

  python tools/trip_kinds.py gpurun_out/r03b/c3_pool.npz [--camera flyover] [--tiles 8]
"""
import argparse
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

F = np.float32
S_MAX = 23


def fbits(x):
    return int(np.array(x, np.float32).view(np.int32))


def ibits(i):
    return F(np.array(i & 0xFFFFFFFF, np.uint32).view(np.float32))


def hlsl_f2i(x):
    # int <- float conversion of the HLSL float2 stack (round toward zero)
    return int(np.int32(np.float32(x)))


kinds_pop_dist = []   # levels climbed by every POP traced (diagnostics)


def trace_kinds(nodes, o, d):
    """Iteration kinds of one ray (list of str)."""
    ox, oy, oz = F(o[0]) * F(1.0 / 32.0) + F(1.5), F(o[1]) * F(1.0 / 32.0) + F(1.5), F(o[2]) * F(1.0 / 32.0) + F(1.5)
    dx, dy, dz = F(d[0]), F(d[1]), F(d[2])
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        txc, tyc, tzc = F(1.0) / -abs(dx), F(1.0) / -abs(dy), F(1.0) / -abs(dz)
        txb, tyb, tzb = txc * ox, tyc * oy, tzc * oz
        om = 7
        if dx > 0: om ^= 1; txb = F(3.0) * txc - txb
        if dy > 0: om ^= 2; tyb = F(3.0) * tyc - tyb
        if dz > 0: om ^= 4; tzb = F(3.0) * tzc - tzb
        t_min = max(max(F(2.0) * txc - txb, F(2.0) * tyc - tyb), F(2.0) * tzc - tzb)
        t_max = min(min(txc - txb, tyc - tyb), tzc - tzb)
        h = t_max
        t_min = max(t_min, F(0.0))
        stack_p = [0] * 32
        stack_t = [0] * 32
        parent, cd, first, cached, idx = 0, 0, 0, 0, 0
        px = py = pz = F(1.0)
        scale, se = S_MAX - 1, F(0.5)
        if F(1.5) * txc - txb > t_min: idx ^= 1; px = F(1.5)
        if F(1.5) * tyc - tyb > t_min: idx ^= 2; py = F(1.5)
        if F(1.5) * tzc - tzb > t_min: idx ^= 4; pz = F(1.5)
        kinds = []
        while scale < S_MAX:
            if len(kinds) > 65536:
                break
            if not cached:
                n = int(nodes[parent]) if parent < len(nodes) else 0
                cd, first = n & 0xFFFFFFFF, n >> 32
                cached = n != 0
            txk, tyk, tzk = px * txc - txb, py * tyc - tyb, pz * tzc - tzb
            tc_max = min(min(txk, tyk), tzk)
            cm = (cd << (idx ^ om)) & 0xFFFFFFFF
            if (cm & 0x8000) and t_min <= t_max:
                tv_max = min(t_max, tc_max)
                half = se * F(0.5)
                txm, tym, tzm = half * txc + txk, half * tyc + tyk, half * tzc + tzk
                if t_min <= tv_max:
                    if (cm & 0x0080) == 0:
                        kinds.append("HIT")
                        break
                    if tc_max < h:
                        stack_p[scale] = hlsl_f2i(F(parent))
                        stack_t[scale] = hlsl_f2i(F(fbits(t_max)))
                    h = tc_max
                    parent = first + bin(cm & 0x7F).count("1")
                    idx = 0
                    scale -= 1
                    se = half
                    if txm > t_min: idx ^= 1; px = px + se
                    if tym > t_min: idx ^= 2; py = py + se
                    if tzm > t_min: idx ^= 4; pz = pz + se
                    t_max = tv_max
                    cached = 0
                    kinds.append("PUSH")
                    continue
            sm = 0
            if txk <= tc_max: sm ^= 1; px = px - se
            if tyk <= tc_max: sm ^= 2; py = py - se
            if tzk <= tc_max: sm ^= 4; pz = pz - se
            t_min = tc_max
            idx ^= sm
            if idx & sm:
                db = 0
                if sm & 1: db |= fbits(px) ^ fbits(px + se)
                if sm & 2: db |= fbits(py) ^ fbits(py + se)
                if sm & 4: db |= fbits(pz) ^ fbits(pz + se)
                old_scale = scale
                scale = (fbits(F(db)) >> 23) - 127
                kinds_pop_dist.append(scale - old_scale)
                se = ibits((scale - S_MAX + 127) << 23)
                parent = stack_p[scale & 31] & 0xFFFFFFFF
                t_max = ibits(stack_t[scale & 31])
                shx, shy, shz = fbits(px) >> scale, fbits(py) >> scale, fbits(pz) >> scale
                px, py, pz = ibits(shx << scale), ibits(shy << scale), ibits(shz << scale)
                idx = (shx & 1) | ((shy & 1) << 1) | ((shz & 1) << 2)
                h = F(0.0)
                cached = 0
                kinds.append("POP")
            else:
                kinds.append("ADV")
    return kinds


def fold2(ks):
    """Folded trips of one ray when a trip whose iteration is a same-node ADVANCE also
    runs the next iteration (a second evaluation stage, no fetch in between), and
    which of those trips carry the second stage."""
    trips, two = [], []
    i = 0
    while i < len(ks):
        if ks[i] == "ADV" and i + 1 < len(ks):
            two.append(True)
            i += 2
        else:
            two.append(False)
            i += 1
        trips.append(1)
    return two


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--camera", default="flyover")
    ap.add_argument("--tiles", type=int, default=8)
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
    tot = collections.Counter()
    fold2_rows = []
    nodes_l = nodes.tolist()
    for k in order:
        r0, c0 = divmod(int(k), tx)
        per_lane_fold = []
        per_lane_two = []
        kc = collections.Counter()
        for j in range(64):
            y, x = r0 * 8 + j // 8, c0 * 8 + j % 8
            o, d = orc.camera_ray(cam, x, y, W, H)
            ks = trace_kinds(nodes_l, o, d)
            if len(ks) != it[y, x]:
                raise SystemExit(f"restatement disagrees with the oracle at ({x}, {y}): {len(ks)} vs {it[y, x]}")
            kc.update(ks)
            per_lane_fold.append(len(ks) - ks.count("ADV"))
            per_lane_two.append(fold2(ks))
        tot.update(kc)
        f2 = max(len(t) for t in per_lane_two)
        stage2 = sum(1 for j in range(f2) if any(j < len(t) and t[j] for t in per_lane_two))
        fold2_rows.append((int(cost[k]), f2, stage2))
        n = sum(kc.values())
        print(f"tile {int(k):6d} (row {r0}): wave trips {cost[k]:4d}, folded {max(per_lane_fold):4d}   "
              + "  ".join(f"{kk} {100.0 * kc[kk] / n:4.1f}%" for kk in ("PUSH", "ADV", "POP", "HIT")), flush=True)
    for c, f2, st in fold2_rows:
        print(f"two-stage trip: wave trips {c:4d} -> {f2:4d} ({100.0 * f2 / c:5.1f} %), second stage on {st:4d} trips")
    n = sum(tot.values())
    pd = collections.Counter(kinds_pop_dist)
    npd = sum(pd.values())
    print("POP levels climbed: " + "  ".join(f"{k}: {100.0 * v / npd:.1f}%" for k, v in sorted(pd.items())))
    print("all: " + "  ".join(f"{kk} {100.0 * tot[kk] / n:4.1f}%" for kk in ("PUSH", "ADV", "POP", "HIT")))


if __name__ == "__main__":
    main()
