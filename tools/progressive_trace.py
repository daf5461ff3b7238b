"""The C# shim's per-frame call (svo_render_progressive_async, RGB24) alone, for a timeline: a held
view at a fixed offset, a held view jittered every frame, and a pan (a new view every frame), each
`--frames` frames after 30 untimed ones, host clock per frame printed.  Run it under
`rocprofv3 --kernel-trace --memory-copy-trace -f csv` and pass the output directory to --analyse to
split each loop's period into the render stream's kernels, the order builds beside them and the
D2H copy.

  rocprofv3 --kernel-trace --memory-copy-trace -f csv -d gpurun_out/pt -o pt -- python3 tools/progressive_trace.py
  python tools/progressive_trace.py --analyse gpurun_out/pt
"""
import argparse
import csv
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(a):
    import bench
    from raytracingtest_amd import RaytracingMaster, _lib
    from raytracingtest_amd.camera import column_major, jitter_offsets, main_light, pan_cameras
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = bench.CONFIGS["C3"]
    W, H = cfg["width"], cfg["height"]
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    conf = {}
    for kv in a.set:
        k, v = kv.split("=", 1)
        conf[k] = float(v) if "." in v else int(v, 0)
    rm = RaytracingMaster(capacity_nodes=len(svo), config=conf)
    rm.SetSVOBuffer(svo)
    L = _lib.lib()
    n = a.frames + 64
    offs = [(float(x), float(y)) for x, y in jitter_offsets(n)]
    views = [tuple(column_major(m) for m in c.uniforms(W, H)) for c in pan_cameras(a.pose, n)]
    light = np.ascontiguousarray(main_light(), np.float32)
    ptr = ctypes.c_void_p()
    out = {"pose": a.pose, "set": conf or "defaults"}
    for kind in ("warm", "fixed", "jitter", "pan"):
        sample = 0
        frames = 400 if kind == "warm" else a.frames

        def one(k):
            nonlocal sample
            c, p = views[k if kind == "pan" else 0]
            ox, oy = (0.5, 0.5) if kind in ("fixed", "warm") else offs[k]
            _lib.check(L.svo_set_camera(rm._ctx, c.ctypes.data, p.ctypes.data, ox, oy, light.ctypes.data), "camera")
            s = 0 if kind == "pan" else sample
            _lib.check(L.svo_render_progressive_async(rm._ctx, W, H, 0, s, _lib.PIXELS_RGB8, ctypes.byref(ptr)),
                       "svo_render_progressive_async")
            sample = s + 1

        for k in range(30):
            one(k)
        _lib.check(L.svo_progressive_last(rm._ctx, ctypes.byref(ptr)), "last")
        time.sleep(0.002)   # a gap in the timeline between the loops
        t = time.perf_counter()
        for k in range(frames):
            one(k % n)
        _lib.check(L.svo_progressive_last(rm._ctx, ctypes.byref(ptr)), "last")
        if kind != "warm":
            out[kind + "_ms_per_frame"] = round((time.perf_counter() - t) / frames * 1e3, 4)
        time.sleep(0.002)
    rm.close()
    print(json.dumps(out), flush=True)


def analyse(d):
    ktrace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ctrace = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)[0]
    ev = []
    for r in csv.DictReader(open(ktrace)):
        n = r["Kernel_Name"]
        short = ("splat" if "beam_splat" in n else "order" if "order_strips" in n else
                 "render" if "render_" in n else "accumulate" if "accumulate" in n else
                 "pack" if "pack_" in n else None)
        if short:
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
    for r in csv.DictReader(open(ctrace)):
        if "DEVICE_TO_HOST" in r.get("Direction", "") or "D2H" in r.get("Direction", "").upper() or \
                r.get("Kind", "").endswith("DEVICE_TO_HOST"):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "d2h"))
    ev.sort()
    # the loops are separated by the 2 ms host sleeps: split at gaps > 1 ms
    loops, cur = [], [ev[0]]
    for e in ev[1:]:
        if e[0] - max(x[1] for x in cur[-8:]) > 1_000_000:
            loops.append(cur)
            cur = []
        cur.append(e)
    loops.append(cur)
    res = []
    for lp in loops:
        packs = [e for e in lp if e[2] == "pack"]
        if len(packs) < 20:
            continue
        span = (packs[-1][1] - packs[10][1]) / (len(packs) - 11) / 1e3   # us per frame, pack to pack
        per = {}
        for kind in ("splat", "render", "accumulate", "pack", "order", "d2h"):
            ds = [(e[1] - e[0]) / 1e3 for e in lp if e[2] == kind]
            per[kind] = {"n": len(ds), "mean_us": round(float(np.mean(ds)), 2) if ds else 0.0}
        # the render stream's busy time per frame and the copy's
        res.append({"frames": len(packs), "us_per_frame_pack_to_pack": round(span, 2), "kernels": per})
    print(json.dumps(res, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--pose", default="flyover")
    ap.add_argument("--set", action="append", default=[])
    ap.add_argument("--analyse", default=None)
    a = ap.parse_args()
    if a.analyse:
        analyse(a.analyse)
    else:
        run(a)


if __name__ == "__main__":
    main()
