"""Model of lane refill from a wave's own tile list, from the
oracle's per-ray iteration counts (tools/simd_efficiency.py --save-iters).

A wave owns a static list of rays (K 8x8 tiles); it starts with the first 64,
and whenever at least T of its lanes are idle at the end of a trip (and rays
remain) it refills them with the next rays of its list (ballot + mbcnt rank, no
atomics).  Reported per (K, T): total wave trips, refill events, the heaviest
wave's trips (the frame's critical path: one ray's iterations are serial), and
a cost in trip units: trips + R * (refill events + waves), R = one refill's
setup + record + stores in trip-equivalents.

  python tools/refill_model.py gpurun_out/iters_c3_flyover.npz [--r 3]
"""
import argparse

import numpy as np


def tiles(iters, group):
    """Per-ray iteration counts ordered as waves of `group` 8x8 tiles (2x2 or 4x1 blocks)."""
    H, W = iters.shape
    gx, gy = group
    Hp, Wp = -(-H // (8 * gy)) * 8 * gy, -(-W // (8 * gx)) * 8 * gx
    a = np.zeros((Hp, Wp), np.int64)
    a[:H, :W] = iters
    # (by, gy, 8, bx, gx, 8) -> wave (by, bx), then tile (gy, gx), then lane (8, 8)
    a = a.reshape(Hp // (8 * gy), gy, 8, Wp // (8 * gx), gx, 8).transpose(0, 3, 1, 4, 2, 5)
    return a.reshape(-1, gx * gy * 64)


def simulate(q, T):
    """q: (waves, n) ray iteration counts (0 = padding).  Returns per-wave trips and refills."""
    nw, n = q.shape
    lanes = q[:, :64].copy()
    ptr = np.full(nw, 64)
    trips = np.zeros(nw, np.int64)
    refills = np.zeros(nw, np.int64)
    alive = (lanes > 0).any(1) | (ptr < n)
    while alive.any():
        act = lanes > 0
        running = act.any(1)
        trips += running
        lanes = np.where(act, lanes - 1, 0)
        idle = lanes == 0
        n_idle = idle.sum(1)
        left = n - ptr
        do = (n_idle >= np.minimum(T, 64)) & (left > 0)
        do |= (n_idle == 64) & (left > 0)      # an empty wave always refills
        if do.any():
            w = np.nonzero(do)[0]
            rank = np.cumsum(idle[w], 1) - 1      # mbcnt rank among the idle lanes
            take = idle[w] & (rank < left[w, None])
            src = ptr[w, None] + rank
            src = np.where(take, src, 0)
            vals = np.take_along_axis(q[w], np.minimum(src, n - 1), 1)
            lanes[w] = np.where(take, vals, lanes[w])
            ptr[w] += take.sum(1)
            refills[w] += 1
        alive = (lanes > 0).any(1) | (ptr < n)
    return trips, refills


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--r", type=float, default=3.0, help="refill cost in trip units")
    a = ap.parse_args()
    it = np.load(a.npz)["iters"].astype(np.int64)
    base = tiles(it, (1, 1))
    tmax = base.max(1)
    ideal = it.sum() / 64
    print(f"rays {it.size}, iterations {it.sum()}, ideal wave trips {ideal:.0f}")
    print(f"tile kernel (K=1, no refill): trips {tmax.sum()} (eff {ideal / tmax.sum():.3f}), "
          f"heaviest wave {tmax.max()}, cost {tmax.sum() + a.r * len(tmax):.0f}")
    # cost-paired lists: wave i = the i-th heaviest tile + the K-1 lightest remaining
    # (the previous launch's tile costs give the order): keeps the critical path
    c = tmax
    o = np.argsort(-c, kind="stable")
    n = len(o)
    for K in (2, 4):
        m = n // K
        groups = [o[:m]] + [o[n - 1 - np.arange(m) - j * m] for j in range(K - 1)]
        q = np.concatenate([base[g] for g in groups], 1)
        for T in (1, 8, 16):
            tr, rf = simulate(q, T)
            cost = tr.sum() + a.r * (rf.sum() + len(tr))
            print(f"paired K={K} T={T:2d}: trips {tr.sum()} (eff {ideal / tr.sum():.3f}), refills {rf.sum()}, "
                  f"heaviest wave {tr.max()} trips, cost {cost:.0f} ({cost / (tmax.sum() + a.r * len(tmax)):.3f} x)")
    for group in ((2, 1), (2, 2), (4, 2)):
        q = tiles(it, group)
        for T in (8, 16, 32, 48):
            tr, rf = simulate(q, T)
            cost = tr.sum() + a.r * (rf.sum() + len(tr))
            print(f"K={group[0] * group[1]} T={T:2d}: trips {tr.sum()} (eff {ideal / tr.sum():.3f}), refills "
                  f"{rf.sum()}, heaviest wave {tr.max()} trips (+{rf[tr.argmax()]} refills), cost {cost:.0f} "
                  f"({cost / (tmax.sum() + a.r * len(tmax)):.3f} x tile kernel)")


if __name__ == "__main__":
    main()
