"""Tile dispatch-order experiments (diagnostics; placement only, results are
identical for every order).

1. per-tile trip counts from one unordered launch (tools/wave_log.py);
2. candidate orders built on the host and written as uint32 permutations;
3. bench.py once per order through SVO_ORDER_FILE (svo_rt.hip reads it).

  python tools/order_experiment.py
"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out", "order_exp")
W, H = 1920, 1080
TX, TY = W // 8, H // 8


def run(cmd, env=None):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run(cmd, cwd=ROOT, env=e, check=True, capture_output=True, text=True, timeout=400).stdout


def morton2(x, y):
    def spread(v):
        v = v.astype(np.uint64)
        out = np.zeros_like(v)
        for b in range(16):
            out |= ((v >> np.uint64(b)) & np.uint64(1)) << np.uint64(2 * b)
        return out
    return spread(x) | (spread(y) << np.uint64(1))


def classes(cost):
    mx = cost.max()
    return np.where(2 * cost >= mx, 0, np.where(4 * cost >= mx, 1, np.where(8 * cost >= mx, 2, 3)))


def interleave(regions):
    """regions: list of 8 tile lists; block b -> region b % 8 while all last."""
    out = []
    k = 0
    while any(k < len(r) for r in regions):
        for r in regions:
            if k < len(r):
                out.append(r[k])
        k += 1
    return np.array(out, np.uint32)


def xcd_regions(cost, key, within):
    seq = np.argsort(key, kind="stable")
    c = np.cumsum(cost[seq].astype(np.float64))
    reg = np.minimum((8 * (c - cost[seq] / 2) / c[-1]).astype(int), 7)
    regions = []
    for x in range(8):
        t = seq[reg == x]
        regions.append(t[within(cost[t])])
    return interleave(regions)


def main():
    os.makedirs(OUT, exist_ok=True)
    log = os.path.join(OUT, "wave_log_unordered.bin")
    run([sys.executable, "tools/wave_log.py", "--out", log], {"SVO_TILE_ORDER": "0"})
    rec = np.fromfile(log, np.uint32).reshape(-1, 8)[: TX * TY]
    cost = (rec[:, 3] >> 8).astype(np.int64)
    tx, ty = np.arange(TX * TY) % TX, np.arange(TX * TY) // TX
    desc = lambda c: np.argsort(-c, kind="stable")
    by_class = lambda c: np.argsort(classes(c), kind="stable")
    orders = {
        "identity": np.arange(TX * TY, dtype=np.uint32),
        "class4": np.argsort(classes(cost), kind="stable").astype(np.uint32),
        "sorted": desc(cost).astype(np.uint32),
        "xcd_rows_sorted": xcd_regions(cost, ty * TX + tx, desc),
        "xcd_morton_sorted": xcd_regions(cost, morton2(tx, ty), desc),
        "xcd_morton_class4": xcd_regions(cost, morton2(tx, ty), by_class),
    }
    res = {}
    for name, o in orders.items():
        assert np.array_equal(np.sort(o), np.arange(TX * TY))
        f = os.path.join(OUT, name + ".u32")
        o.astype(np.uint32).tofile(f)
        ms = []
        for _ in range(2):
            out = run([sys.executable, "bench.py", "--steps", "40", "--warmup", "5", "--cpu-seconds", "0"],
                      {"SVO_ORDER_FILE": f})
            ms.append(json.loads(out.strip().splitlines()[-1])["roofline"]["kernel_ms"])
        res[name] = ms
        print(name, ms, flush=True)
    json.dump(res, open(os.path.join(OUT, "results.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
