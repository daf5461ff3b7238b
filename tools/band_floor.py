"""Where an N-GPU band's time goes: the C3 frame's round-robin 8-row band of
every rank of an N-way split rendered alone on this GPU (the launch each GPU of the split runs), its
GPU time per launch (event span over back-to-back launches, as bench.py's strong_split_rehearsal),
then one launch of the slowest rank's band with the per-workgroup log (SVO_WAVE_LOG: entry, trace
start, trace end, trips, order entry; svo_kernel.hip seg_log / render_tile_kernel) decomposed into
  ramp      first workgroup's entry -> the heaviest wave's entry (dispatch order and CU slots),
  setup     the heaviest wave's entry -> its trace start (order read, camera ray, starts),
  chain     the heaviest wave's trace,
  after     its trace end -> the last trace end of the launch,
and the launch's GPU time beside them (the rest: the dispatch before the first workgroup runs, the
outputs after the last trace, the drain).  100 MHz clock (s_memrealtime).

  python tools/band_floor.py [--gpus 8] [--pose flyover] [--out gpurun_out/band_floor.json] [--set k=v]
  rocprofv3 --kernel-trace --stats -d gpurun_out/band -o band -- python3 tools/band_floor.py --trace-only
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
WORDS = 12   # svo_traverse.h WAVE_LOG_WORDS


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--pose", default="flyover")
    ap.add_argument("--out", default=None)
    ap.add_argument("--timed", type=int, default=150)
    ap.add_argument("--trace-only", action="store_true",
                    help="only the slowest band's launches (30 warmup + --timed), for a rocprofv3 kernel trace")
    ap.add_argument("--rank", type=int, default=-1, help="the band to trace (default: measure, take the slowest)")
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args()
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = CONFIGS["C3"]
    W, H = cfg["width"], cfg["height"]
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    conf = {}
    for kv in a.set:
        k, v = kv.split("=", 1)
        conf[k] = float(v) if "." in v else int(v, 0)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    hits = torch.empty(W * H * 24, dtype=torch.uint8, device=dev)
    rgba = torch.empty(W * H * 16, dtype=torch.uint8, device=dev)

    def make():
        m = RaytracingMaster(capacity_nodes=len(svo), config=conf)
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(CAMERAS[a.pose](), W, H)
        return m

    def band_ms(m, band, timed):
        for _ in range(30):
            m.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), band=band, stream=s.cuda_stream)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(timed):
            m.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), band=band, stream=s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / timed

    m = make()
    for _ in range(400):   # past the clock ramp
        m.render_frame(W, H, hits=hits.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize(dev)
    N = a.gpus
    if a.trace_only:
        band_ms(m, (8, max(a.rank, 0), N), a.timed)
        m.close()
        return
    frame = band_ms(m, None, a.timed)
    per = [band_ms(m, (8, r, N), a.timed) for r in range(N)]
    slow = int(np.argmax(per)) if a.rank < 0 else a.rank
    m.close()
    # one logged launch of the slowest band (a context created with the log switch on)
    log = os.path.abspath(os.path.join(ROOT, "gpurun_out", f"band_floor_wave_log_{N}.bin"))
    os.makedirs(os.path.dirname(log), exist_ok=True)
    os.environ["SVO_WAVE_LOG"] = log
    ml = make()
    del os.environ["SVO_WAVE_LOG"]
    band = (8, slow, N)
    for _ in range(30):   # the order and its segmented parts settle; the last launch's log is kept
        ml.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), band=band, stream=s.cuda_stream)
    torch.cuda.synchronize(dev)
    logged_ms = band_ms(ml, band, 1)
    ml.close()
    rec = np.fromfile(log, np.uint32).reshape(-1, WORDS).astype(np.int64)
    entry, t0, t1, code, trips, ex = rec[:, 8], rec[:, 0], rec[:, 1], rec[:, 2], rec[:, 3] >> 8, rec[:, 9]
    traced = (t1 > 0) & (t0 > 0)
    base = entry[entry > 0].min()
    ent, st, en = entry - base, t0 - base, t1 - base
    dur = np.where(traced, en - st, 0)
    k = int(np.argmax(dur))
    tick = 0.01   # us per s_memrealtime tick (100 MHz)
    out = {
        "pose": a.pose, "frame": f"{W}x{H}", "n_gpus": N, "frame_ms": round(frame, 4),
        "band_ms_per_rank": [round(x, 4) for x in per], "slowest_rank": slow,
        "predicted_speedup": round(frame / max(per), 3), "config": conf or "defaults",
        "logged_launch": {
            "gpu_ms": round(logged_ms, 4),
            "workgroups": int(len(rec)), "traced_workgroups": int(traced.sum()),
            "empty_slots": int(((code & 0xFFFFFFFF) == 0xFFFFFFFF).sum()),
            "part_workgroups": int(((code >> 28) > 0).sum() - ((code & 0xFFFFFFFF) == 0xFFFFFFFF).sum()),
            "first_to_last_trace_end_us": round(en[traced].max() * tick, 2),
            "first_to_last_exit_us": round((ex[traced & (ex > 0)] - base).max() * tick, 2) if (traced & (ex > 0)).any() else None,
            "latest_exit": {"order_entry": hex(int(code[int(np.argmax(np.where(traced & (ex > 0), ex, 0)))])),
                            "trips": int(trips[int(np.argmax(np.where(traced & (ex > 0), ex, 0)))]),
                            "entry_us": round(float(ent[int(np.argmax(np.where(traced & (ex > 0), ex, 0)))]) * tick, 2)},
            "heaviest": {"order_entry": hex(int(code[k])), "trips": int(trips[k]),
                         "ramp_us": round(ent[k] * tick, 2), "setup_us": round((st[k] - ent[k]) * tick, 2),
                         "chain_us": round(dur[k] * tick, 2),
                         "after_us": round((en[traced].max() - en[k]) * tick, 2)},
            "median_setup_us": round(float(np.median(st[traced] - ent[traced])) * tick, 2),
            "median_trace_us": round(float(np.median(dur[traced])) * tick, 2),
            "waves_by_trace_us": {f"<={b}": int((dur[traced] * tick <= b).sum()) for b in (2, 5, 10, 20, 40)},
            "note": "ticks of s_memrealtime; gpu_ms is the same launch's event time (one launch, clock "
                    "ramped); the wave log's stamps add a few instructions per workgroup"},
    }
    js = json.dumps(out)
    print(js, flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(js + "\n")


if __name__ == "__main__":
    main()
