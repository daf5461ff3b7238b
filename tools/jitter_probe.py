"""Why a jittered frame loop renders slower than the repeated (0.5, 0.5) frame:
the C3 render kernel (render_device, value's outputs, span per launch over back-to-back launches)
under pixel-offset sequences that separate the ray set from the staleness of per-stream state:
  fixed(a, b)   the same offset every frame, for several offsets (is the (0.5, 0.5) ray set special?),
  nudge         (0.5, 0.5) and its next float alternating: the jittered-launch policy on an unchanged ray set,
  alt           two offsets alternating (every frame's stored starts and costs are the other ray set's),
  random        a new seeded offset every frame (the drop-in's loop),
and for `random` the per-launch kernel times (library events) against the offsets.

  python tools/jitter_probe.py [--poses flyover,main] [--frames 300] [--set field=value ...]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--poses", default="flyover,main")
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args()
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster, _lib
    from raytracingtest_amd.camera import CAMERAS, column_major, jitter_offsets, main_light
    cfg = CONFIGS["C3"]
    W, H = cfg["width"], cfg["height"]
    from raytracingtest_amd.native_builder import build_sampler_svo
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    conf = {}
    for kv in a.set:
        k, v = kv.split("=", 1)
        conf[k] = float(v) if "." in v else int(v, 0)
    rm = RaytracingMaster(capacity_nodes=len(svo), config=conf)
    rm.SetSVOBuffer(svo)
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    hits = torch.empty(W * H * 24, dtype=torch.uint8, device=dev)
    rgba = torch.empty(W * H * 4, dtype=torch.float32, device=dev)
    light = np.ascontiguousarray(main_light(), np.float32)
    rnd = jitter_offsets(a.frames + 64)
    for pose in a.poses.split(","):
        c2w, ip = CAMERAS[pose]().uniforms(W, H)
        c, p = column_major(c2w), column_major(ip)

        def run(offs, timed=True):
            def one(k):
                ox, oy = offs[k % len(offs)]
                L.svo_set_camera(rm._ctx, c.ctypes.data, p.ctypes.data, float(ox), float(oy), light.ctypes.data)
                rm.render_device(W, H, rgba_ptr=rgba.data_ptr(), hits_ptr=hits.data_ptr(), stream=s.cuda_stream)
            for k in range(40):
                one(k)
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for k in range(a.frames):
                one(k)
                if k == 0:
                    e0.record(s)
            e1.record(s)
            torch.cuda.synchronize(dev)
            return e0.elapsed_time(e1) / (a.frames - 1)

        L.svo_set_camera(rm._ctx, c.ctypes.data, p.ctypes.data, 0.5, 0.5, light.ctypes.data)
        for _ in range(400):   # past the clock ramp
            rm.render_device(W, H, hits_ptr=hits.data_ptr(), stream=s.cuda_stream)
        torch.cuda.synchronize(dev)
        out = {"pose": pose, "set": conf or "defaults"}
        for name, offs in (("fixed_0.5_0.5", [(0.5, 0.5)]), ("fixed_0.1_0.1", [(0.1, 0.1)]),
                           ("fixed_0.9_0.3", [(0.9, 0.3)]), ("fixed_0.25_0.75", [(0.25, 0.75)]),
                           # the same rays every frame, but a "new" offset (one ulp apart) each frame: the
                           # launch is a jittered one (even segment splits), the order's costs are its own
                           ("nudge_0.5", [(0.5, 0.5), (float(np.nextafter(np.float32(0.5), np.float32(1))), 0.5)]),
                           ("alt_0.5_0.1", [(0.5, 0.5), (0.1, 0.1)]), ("random", [tuple(x) for x in rnd]),
                           ("fixed_0.5_0.5_again", [(0.5, 0.5)])):
            out[name] = round(run(offs), 4)
        # per-launch kernel times of the random sequence (library events), against the offsets
        rm.set_kernel_timing(True)
        rm.stage_times()
        for k in range(a.frames):
            ox, oy = rnd[k]
            L.svo_set_camera(rm._ctx, c.ctypes.data, p.ctypes.data, float(ox), float(oy), light.ctypes.data)
            rm.render_device(W, H, rgba_ptr=rgba.data_ptr(), hits_ptr=hits.data_ptr(), stream=s.cuda_stream)
        t = rm.stage_times()
        rm.set_kernel_timing(False)
        q = np.percentile(t, [0, 10, 50, 90, 100])
        out["random_events_ms_pctl_0_10_50_90_100"] = [round(float(x), 4) for x in q]
        out["random_events_every_32nd_mean_ms"] = round(float(np.mean(t[::32])), 4)
        print(json.dumps(out), flush=True)
    rm.close()


if __name__ == "__main__":
    main()
