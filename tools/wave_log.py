"""Per-wave timing of one render of the bench workload (diagnostics).

Runs the tile kernel once with SVO_WAVE_LOG set (svo_rt.hip writes, per wave:
s_memrealtime at trace start / end (100 MHz), HW_ID, XCC_ID | trip count << 8)
and prints the kernel span, the wave-duration distribution, the mean number
of resident waves over the span and a coarse occupancy timeline.

  python tools/wave_log.py [--config C3] [--camera flyover] [--tile-row N | -2]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORDS = 12   # svo_traverse.h WAVE_LOG_WORDS
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3", help="bench.py CONFIGS entry: frame size, pool, stack mode")
    ap.add_argument("--camera", default=None, help="default: the config's camera")
    ap.add_argument("--max-level", type=int, default=None)
    ap.add_argument("--out", default="gpurun_out/wave_log.bin")
    ap.add_argument("--tile-row", type=int, default=-1,
                    help="render only this 8-row band (a near-empty GPU); -2: the band holding the frame's "
                         "heaviest tile (found from a logged full-frame launch first)")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    os.environ["SVO_WAVE_LOG"] = os.path.abspath(args.out)
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo

    cfg = CONFIGS[args.config]
    W, H = cfg["width"], cfg["height"]
    mode = cfg["stack_mode"]
    svo = build_sampler_svo(4, args.max_level or cfg["max_level"])
    rm = RaytracingMaster(capacity_nodes=len(svo))
    rm.SetSVOBuffer(svo)
    rm.UpdateShaderParameters(CAMERAS[args.camera or cfg["camera"]](), W, H)
    hits = torch.empty(W * H * 24, dtype=torch.uint8, device="cuda")
    rgba = torch.empty(W * H * 4, dtype=torch.float32, device="cuda")
    if args.tile_row == -2:
        for _ in range(3):
            rm.render_device(W, H, rgba.data_ptr(), hits.data_ptr(), stack_mode=mode)
        rm.synchronize()
        full = np.fromfile(args.out, np.uint32).reshape(-1, WORDS)
        k = int(np.argmax(full[:, 3] >> 8))
        args.tile_row = int(full[k, 2]) // ((W + 7) // 8)
        print(f"heaviest tile {int(full[k, 2])}: {int(full[k, 3] >> 8)} trips, tile row {args.tile_row}")
    band = None if args.tile_row < 0 else (8, args.tile_row, (H + 7) // 8)
    for _ in range(3):
        rm.render_device(W, H, rgba.data_ptr(), hits.data_ptr(), band=band, stack_mode=mode)
    rm.synchronize()
    # uninstrumented timing of the same launch (the log is only taken while SVO_WAVE_LOG is set)
    del os.environ["SVO_WAVE_LOG"]
    s = torch.cuda.Stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for a, b in evs:
        a.record(s)
        rm.render_device(W, H, rgba.data_ptr(), hits.data_ptr(), band=band, stack_mode=mode, stream=s.cuda_stream)
        b.record(s)
    torch.cuda.synchronize()
    print(f"uninstrumented launch: {np.median([a.elapsed_time(b) for a, b in evs]) * 1e3:.1f} us (median of 10)")
    log = np.fromfile(args.out, np.uint32).reshape(-1, WORDS)
    log = log[(log[:, 0] != 0) | (log[:, 1] != 0)]
    t0 = log[:, 0].astype(np.int64)
    t1 = log[:, 1].astype(np.int64)
    t1 = np.where(t1 < t0, t1 + (1 << 32), t1)
    base = t0.min()
    t0 -= base
    t1 -= base
    dur = (t1 - t0) * 10e-3    # us
    trips = log[:, 3] >> 8
    span = t1.max() * 10e-3
    print(f"waves {len(log)}  span {span:.1f} us  (100 MHz clock)")
    q = np.percentile(dur, [0, 10, 50, 90, 99, 100])
    print("wave duration us  min/p10/p50/p90/p99/max", np.round(q, 2))
    q = np.percentile(trips, [0, 10, 50, 90, 99, 100])
    print("trips             min/p10/p50/p90/p99/max", q)
    print(f"sum of wave time {dur.sum():.0f} us -> mean resident waves {dur.sum() / span:.0f}"
          f" (chip max 256 CUs x 32 = 8192)")
    # resident-wave timeline (20 bins)
    nb = 20
    edges = np.linspace(0, t1.max(), nb + 1)
    res = []
    for a, b in zip(edges[:-1], edges[1:]):
        ov = np.clip(np.minimum(t1, b) - np.maximum(t0, a), 0, None).sum() / (b - a)
        res.append(ov)
    print("resident waves per 5% of span:", " ".join(f"{int(v)}" for v in res))
    # start times: how fast the dispatcher issues
    ts = np.sort(t0) * 10e-3
    print("wave starts by t(us): 25%/50%/75%/100% of waves started at",
          np.round([ts[int(len(ts) * f) - 1] for f in (0.25, 0.5, 0.75, 1.0)], 1))
    # duration vs screen position (block order = row-major tiles)
    ntx = W // 8
    ty = np.arange(len(log)) // ntx
    if ty.max() >= 15:
        rows = [dur[ty == y].mean() for y in range(0, ty.max() + 1, 15)]
        print("mean wave us per 15 tile-rows (top->bottom):", " ".join(f"{v:.1f}" for v in rows))
    # instrumented loop (s_memtime shader cycles): where the heavy waves spend their trips
    loop_c = log[:, 4].astype(np.float64)
    fetch_c = log[:, 5].astype(np.float64)
    ft = log[:, 6].astype(np.float64)
    pt = log[:, 7].astype(np.float64)
    heavy = trips >= np.percentile(trips, 99)
    push_only = log[:, 5].astype(np.int64) & 0xFFFF
    adv_only = log[:, 5].astype(np.int64) >> 16
    for name, m in (("all", np.ones(len(trips), bool)), ("top 1% trips", heavy)):
        tr = trips[m].sum()
        print(f"{name}: cycles/trip {loop_c[m].sum() / tr:.0f}, fetching trips {ft[m].sum() / tr:.2f},"
              f" popping trips {pt[m].sum() / tr:.2f}, push-only trips {push_only[m].sum() / tr:.2f},"
              f" advance-only trips {adv_only[m].sum() / tr:.2f}")
    # the whole wave (entry .. its stores issued) against the traced loop
    te = log[:, 8].astype(np.int64)
    tx = log[:, 9].astype(np.int64)
    ok = (te != 0) & (tx != 0)
    if ok.any():
        te = np.where(te > log[:, 0], te - (1 << 32), te) - base
        tx = np.where(tx < log[:, 1], tx + (1 << 32), tx) - base
        setup = (t0 - te)[ok] * 10e-3
        rec = (tx - t1)[ok] * 10e-3
        whole = (tx - te)[ok] * 10e-3
        q = [0, 10, 50, 90, 99, 100]
        print("setup us (entry -> loop)      min/p10/p50/p90/p99/max", np.round(np.percentile(setup, q), 2))
        print("record us (loop -> stores)    min/p10/p50/p90/p99/max", np.round(np.percentile(rec, q), 2))
        print(f"whole waves: sum {whole.sum():.0f} us -> mean resident {whole.sum() / ((tx.max() - te.min()) * 10e-3):.0f};"
              f" setup {setup.sum() / whole.sum():.1%}, record {rec.sum() / whole.sum():.1%} of wave time;"
              f" span {(tx.max() - te.min()) * 10e-3:.1f} us")
        nb = 20
        lo, hi = te[ok].min(), tx[ok].max()
        edges = np.linspace(lo, hi, nb + 1)
        res = [np.clip(np.minimum(tx[ok], b) - np.maximum(te[ok], a), 0, None).sum() / (b - a)
               for a, b in zip(edges[:-1], edges[1:])]
        print("resident whole waves per 5% of span:", " ".join(f"{int(v)}" for v in res))
    hw = log[:, 10].astype(np.int64)
    if hw.any():   # gfx9 HW_ID: wave_id [3:0], simd_id [5:4], cu_id [11:8], sh_id [12], se_id [15:13]
        cu = ((log[:, 3] & 0xFF).astype(np.int64) << 8) | ((hw >> 13) & 7) << 5 | ((hw >> 12) & 1) << 4 | ((hw >> 8) & 15)
        ucu, cnt = np.unique(cu, return_counts=True)
        simd = (hw >> 4) & 3
        print(f"distinct CUs used {len(ucu)}; waves per CU min/median/max {cnt.min()}/{int(np.median(cnt))}/{cnt.max()};"
              f" SIMD ids seen {np.unique(simd).tolist()}; wave ids seen {np.unique(hw & 15).tolist()}")
        if ok.any():   # peak concurrent whole waves on one CU
            peak = 0
            for c in ucu[:64]:
                m = ok & (cu == c)
                ev = np.concatenate([np.stack([te[m], np.ones(m.sum(), np.int64)], 1),
                                     np.stack([tx[m], -np.ones(m.sum(), np.int64)], 1)])
                ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
                peak = max(peak, int(np.cumsum(ev[:, 1]).max()))
            print(f"peak concurrent waves on one CU (first 64 CUs): {peak}")
    xcc = log[:, 3] & 0xFF
    print("waves per XCC:", np.bincount(xcc, minlength=8)[:8])
    for x in range(8):
        m = xcc == x
        print(f"  xcc {x}: busy-sum {dur[m].sum():.0f} us, last end {t1[m].max() * 10e-3:.1f} us")


if __name__ == "__main__":
    main()
