"""Per-launch render-kernel durations and the shader clock beside them (VERDICT r3
item 1: why the driver's K = 20 bench reads a slower kernel than K = 1000 runs).

Phases, one process, the C3 pool built exactly as bench.py builds it:
  driver   bench.py's own sequence at --gpus 1 --steps 20 --warmup 5 (build, upload,
           instrumented count, 5 warmup, host copy of the records, 20 + 20 launches),
           then more launches at the same view up to --launches
  idle     the host sleeps --idle-s (GPU idle), then --short launches at the same view
  newview  --short launches at the overview pose, then --short at flyover again (a new
           view on a hot GPU), then the same two once more (revisits)
Every launch's kernel is bracketed by the library's events (svo_stage_times); a
one-wave sampler on a second stream stamps (s_memrealtime, s_memtime) every 10 us
through each phase, so each launch gets the shader clock it ran at.

  python tools/launch_series.py [--launches 1500] > gpurun_out/series.json
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SAMPLER = os.path.join(ROOT, "tools", "build", "libclock_sampler.so")


class Sampler:
    def __init__(self, torch, dev, n):
        self.torch, self.n = torch, n
        self.L = ctypes.CDLL(SAMPLER)
        self.L.clock_sampler_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.c_void_p]
        self.buf = torch.zeros(2 * n, dtype=torch.int64, device=dev)
        self.stream = torch.cuda.Stream(dev)

    def start(self, interval_ticks=1000):
        """Start sampling; self.ev marks the start on the sampler's stream (launch start
        times are taken relative to it, so both series share one time axis)."""
        self.buf.zero_()
        self.torch.cuda.synchronize()
        self.ev = self.torch.cuda.Event(enable_timing=True)
        self.ev.record(self.stream)
        rc = self.L.clock_sampler_launch(self.buf.data_ptr(), self.n, interval_ticks, self.stream.cuda_stream)
        if rc:
            raise RuntimeError(f"clock sampler launch: {rc}")

    def read(self):
        """(t_us since the first sample, clock MHz) per interval."""
        self.stream.synchronize()
        a = self.buf.cpu().numpy().view(np.uint64).reshape(-1, 2).astype(np.float64)
        a = a[a[:, 0] > 0]
        rt, st = a[:, 0], a[:, 1]
        mhz = np.diff(st) / np.maximum(np.diff(rt), 1) * 100.0
        return (rt[1:] - rt[0]) / 100.0, mhz


def windows(x, edges):
    out = []
    for a, b in zip(edges[:-1], edges[1:]):
        if a < len(x):
            seg = x[a:min(b, len(x))]
            out.append({"launches": f"{a}-{min(b, len(x)) - 1}", "mean": round(float(np.mean(seg)), 5),
                        "median": round(float(np.median(seg)), 5), "min": round(float(np.min(seg)), 5),
                        "max": round(float(np.max(seg)), 5)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=1500)
    ap.add_argument("--short", type=int, default=200)
    ap.add_argument("--idle-s", type=float, default=1.0)
    a = ap.parse_args()
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = CONFIGS["C3"]
    W, H = cfg["width"], cfg["height"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sampler = Sampler(torch, dev, 60000)
    out = {"workload": "C3 1920x1080 flyover (bench.py's default), per-launch primary-kernel ms"}

    t0 = time.time()
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"], device=0)
    rm = RaytracingMaster(device=0, capacity_nodes=len(svo))
    rm.SetSVOBuffer(svo)
    rm.UpdateShaderParameters(CAMERAS["flyover"](), W, H)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    hits = torch.empty(W * H * 24, dtype=torch.uint8, device=dev)
    rgba = torch.empty(W * H * 4, dtype=torch.float32, device=dev)
    out["build_s"] = round(time.time() - t0, 2)

    def launch():
        rm.render_device(W, H, rgba_ptr=rgba.data_ptr(), hits_ptr=hits.data_ptr(), stack_mode=0, stream=sptr)

    def run(n, marks, first=0):
        """n launches; a timing event on the render stream every 10 launches (the
        launch's start time on the sampler's time axis, us)."""
        evs = []
        for i in range(n):
            if i % 10 == 0:
                e = torch.cuda.Event(enable_timing=True)
                e.record(stream)
                evs.append((first + i, e))
            launch()
        stream.synchronize()   # the render stream only: a device-wide sync would wait for the sampler
        marks.extend((i, sampler.ev.elapsed_time(e) * 1e3) for i, e in evs)

    def clock_at(marks, t_us, mhz, n):
        """shader clock (median of the samples in [start of launch i, start of launch i + 10))."""
        res = []
        for j, (i, ts) in enumerate(marks):
            te = marks[j + 1][1] if j + 1 < len(marks) else ts + 1e3
            sel = (t_us >= ts) & (t_us < te)
            res.append((i, round(float(np.median(mhz[sel])), 1) if sel.any() else None))
        return res

    # ---- driver: bench.py's sequence (count, 5 warmup, host copy, 20 timed, 20 kernel-timed, ...)
    rm.set_kernel_timing(True)
    rm.kernel_time()
    sampler.start()
    fetch = torch.zeros(W * H, dtype=torch.int32, device=dev)
    marks = []
    rm.count_fetches_device(W, H, fetch.data_ptr(), stack_mode=0, stream=sptr)
    run(5, marks)
    _ = hits.cpu()          # bench.py's host copy of the records after the warmup (render stream)
    run(a.launches - 5, marks, first=5)
    seq = rm.stage_times()
    t_us, mhz = sampler.read()
    out["driver"] = {"kernel_ms": [round(float(x), 5) for x in seq],
                     "windows_ms": windows(seq, [0, 5, 25, 45, 100, 200, 400, 700, 1000, 1500, 3000]),
                     "sampler_span_us": round(float(t_us[-1]), 1) if len(t_us) else None,
                     "clock_mhz_per_10_launches": clock_at(marks, t_us, mhz, len(seq)),
                     "bench_kernel_ms_equivalent": round(float(np.mean(seq[25:45])), 5),
                     "k1000_equivalent": round(float(np.mean(seq[50:1050])), 5) if len(seq) >= 1050 else None}

    # ---- idle: the GPU sits idle, then the same view again
    time.sleep(a.idle_s)
    sampler.start()
    marks = []
    run(a.short, marks)
    seq = rm.stage_times()
    t_us, mhz = sampler.read()
    out["idle"] = {"idle_s": a.idle_s, "kernel_ms": [round(float(x), 5) for x in seq],
                   "windows_ms": windows(seq, [0, 5, 10, 20, 50, 100, 200, 400]),
                   "clock_mhz_per_10_launches": clock_at(marks, t_us, mhz, len(seq))}

    # ---- newview: overview, flyover, overview, flyover on a hot GPU
    out["newview"] = []
    for pose in ("overview", "flyover", "overview", "flyover", "main", "flyover"):
        rm.UpdateShaderParameters(CAMERAS[pose](), W, H)
        sampler.start()
        marks = []
        run(a.short, marks)
        seq = rm.stage_times()
        t_us, mhz = sampler.read()
        out["newview"].append({"pose": pose, "kernel_ms": [round(float(x), 5) for x in seq],
                               "windows_ms": windows(seq, [0, 1, 2, 5, 10, 20, 50, 100, 200, 400]),
                               "clock_mhz_per_10_launches": clock_at(marks, t_us, mhz, len(seq))})
    rm.set_kernel_timing(False)
    rm.close()
    print(json.dumps(out))
    # a short human summary on stderr
    print("driver windows:", json.dumps(out["driver"]["windows_ms"]), file=sys.stderr)
    print("driver clock:", out["driver"]["clock_mhz_per_10_launches"][:40], file=sys.stderr)
    print("idle windows:", json.dumps(out["idle"]["windows_ms"]), file=sys.stderr)
    print("idle clock:", out["idle"]["clock_mhz_per_10_launches"][:20], file=sys.stderr)
    for r in out["newview"]:
        print(r["pose"], json.dumps(r["windows_ms"]), r["clock_mhz_per_10_launches"][:6], file=sys.stderr)


if __name__ == "__main__":
    main()
