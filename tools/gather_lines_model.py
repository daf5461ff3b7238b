"""How many distinct 128-byte lines one trip's node gather touches, under other node layouts.
tools/gather_latency.hip puts a lone wave64 gather of 8-byte words at ~136 cycles (L1) when its
lanes touch <= 4 lines and ~190-200 when they touch 16-64; the bench kernel's gathers touch ~27
(PMC: 28.4 M L1 accesses over 1.07 M wave loads).  This model counts the lines per wave trip of
the heaviest C3 tiles and of a sample of terrain tiles, with the bench kernel's fetch pattern
(every lane loads its current node on every trip, finished lanes their last one), for:

  dfs8  : the pool as uploaded (NaiveCreator.cs:132-193 order, 8-byte V2 nodes)
  bfs8  : the same nodes in breadth-first order (siblings contiguous, cousins adjacent), 8 B
  dfs4  : the uploaded order at a hypothetical 4-byte node width
  bfs4  : breadth-first at 4 bytes

Node indices per lane and iteration come from a float32 restatement of the loop
(NVIDIASVO.compute:57-156, HLSL stack), checked against the oracle's iteration count ray by ray.

  python tools/gather_lines_model.py gpurun_out/r04i/c3_pool.npz [--heavy 16] [--sample 48]
"""
import argparse
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from trip_kinds import F, S_MAX, fbits, ibits, hlsl_f2i  # noqa: E402


def trace_parents(nodes, o, d):
    """The node each iteration of one ray reads (its `parent` at the top of the iteration)."""
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
        seq = []
        while scale < S_MAX and len(seq) <= 65536:
            seq.append(parent)
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
                scale = (fbits(F(db)) >> 23) - 127
                se = ibits((scale - S_MAX + 127) << 23)
                parent = stack_p[scale & 31] & 0xFFFFFFFF
                t_max = ibits(stack_t[scale & 31])
                shx, shy, shz = fbits(px) >> scale, fbits(py) >> scale, fbits(pz) >> scale
                px, py, pz = ibits(shx << scale), ibits(shy << scale), ibits(shz << scale)
                idx = (shx & 1) | ((shy & 1) << 1) | ((shz & 1) << 2)
                h = F(0.0)
                cached = 0
    return seq


def bfs_order(nodes):
    """new index of every node when the pool is laid out breadth-first from the root."""
    lo = (nodes & 0xFFFF).astype(np.int64)
    first = (nodes >> 32).astype(np.int64)
    nonleaf = lo & 0xFF
    cnt = np.array([bin(v).count("1") for v in range(256)], np.int64)[nonleaf]
    new = np.full(len(nodes), -1, np.int64)
    frontier = np.array([0], np.int64)
    nxt = 0
    while len(frontier):
        new[frontier] = np.arange(nxt, nxt + len(frontier))
        nxt += len(frontier)
        c = cnt[frontier]
        f = first[frontier]
        keep = c > 0
        frontier = np.concatenate([np.arange(a, a + k) for a, k in zip(f[keep], c[keep])]) if keep.any() else \
            np.array([], np.int64)
    return new


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--camera", default="flyover")
    ap.add_argument("--heavy", type=int, default=16)
    ap.add_argument("--sample", type=int, default=48)
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
    heavy = list(np.argsort(-cost)[:a.heavy])
    rng = np.random.default_rng(5)
    terrain = np.flatnonzero(cost >= 20)
    sample = list(rng.choice(terrain, size=min(a.sample, len(terrain)), replace=False))
    bfs = bfs_order(nodes)
    assert (bfs >= 0).sum() == len(nodes), "pool is not one tree"
    layouts = {"dfs8": (None, 16), "bfs8": (bfs, 16), "dfs4": (None, 32), "bfs4": (bfs, 32)}
    nodes_l = nodes.tolist()
    for name, tl in (("heaviest", heavy), ("terrain sample", sample)):
        tot = collections.Counter()
        trips = 0
        for k in tl:
            r0, c0 = divmod(int(k), tx)
            seqs = []
            for j in range(64):
                y, x = r0 * 8 + j // 8, c0 * 8 + j % 8
                o, d = orc.camera_ray(cam, x, y, W, H)
                s = trace_parents(nodes_l, o, d)
                if len(s) != it[y, x]:
                    raise SystemExit(f"restatement disagrees with the oracle at ({x}, {y}): {len(s)} vs {it[y, x]}")
                seqs.append(np.array(s, np.int64))
            n = max(len(s) for s in seqs)
            # wave trip t: every lane's node (a finished lane keeps re-loading its last one)
            m = np.stack([np.concatenate([s, np.full(n - len(s), s[-1])]) for s in seqs])   # 64 x n
            trips += n
            for lname, (perm, per_line) in layouts.items():
                idx = m if perm is None else perm[m]
                lines = idx // per_line
                tot[lname] += sum(len(np.unique(lines[:, t])) for t in range(n))
        print(f"{name} ({len(tl)} tiles, {trips} wave trips): distinct 128-B lines per wave trip  " +
              "  ".join(f"{k} {tot[k] / trips:5.2f}" for k in layouts), flush=True)


if __name__ == "__main__":
    main()
