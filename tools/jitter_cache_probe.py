"""The L2 behaviour of a jittered frame against the repeated one: the C3 render at
a held view, `--launches` at the fixed (0.5, 0.5) offset, then as many with a new seeded offset each,
then the fixed offset again -- run under `rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace`;
--analyse splits the per-dispatch counters by phase (dispatch order).

  rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --kernel-include-regex render_seg_kernel \\
      -d gpurun_out/jc -o jc -f csv -- python3 tools/jitter_cache_probe.py
  python tools/jitter_cache_probe.py --analyse gpurun_out/jc --launches 200
"""
import argparse
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(a):
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster, _lib
    from raytracingtest_amd.camera import CAMERAS, column_major, jitter_offsets, main_light
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = CONFIGS["C3"]
    W, H = cfg["width"], cfg["height"]
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    rm = RaytracingMaster(capacity_nodes=len(svo))
    rm.SetSVOBuffer(svo)
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    hits = torch.empty(W * H * 24, dtype=torch.uint8, device=dev)
    rgba = torch.empty(W * H * 4, dtype=torch.float32, device=dev)
    c2w, ip = CAMERAS[a.pose]().uniforms(W, H)
    c, p = column_major(c2w), column_major(ip)
    light = np.ascontiguousarray(main_light(), np.float32)
    offs = jitter_offsets(a.launches + 8)

    def one(ox, oy):
        L.svo_set_camera(rm._ctx, c.ctypes.data, p.ctypes.data, float(ox), float(oy), light.ctypes.data)
        rm.render_device(W, H, rgba_ptr=rgba.data_ptr(), hits_ptr=hits.data_ptr(), stream=s.cuda_stream)

    for _ in range(a.warm):
        one(0.5, 0.5)
    for _ in range(a.launches):
        one(0.5, 0.5)
    for k in range(a.launches):
        one(*offs[k])
    for _ in range(a.launches):
        one(0.5, 0.5)
    torch.cuda.synchronize(dev)
    rm.close()


def analyse(a):
    f = glob.glob(os.path.join(a.analyse, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        per.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(per)
    ids = ids[-3 * a.launches:]   # the three phases (the warm-up launches before them)
    out = {}
    for i, name in enumerate(("fixed", "jittered", "fixed_again")):
        ph = [per[d] for d in ids[i * a.launches:(i + 1) * a.launches]]
        hit = np.mean([x.get("TCC_HIT_sum", 0) for x in ph])
        miss = np.mean([x.get("TCC_MISS_sum", 0) for x in ph])
        out[name] = {"launches": len(ph), "tcc_hit": round(float(hit)), "tcc_miss": round(float(miss)),
                     "l2_hit_rate": round(float(hit / (hit + miss)), 4)}
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pose", default="flyover")
    ap.add_argument("--launches", type=int, default=200)
    ap.add_argument("--warm", type=int, default=100)
    ap.add_argument("--analyse", default=None)
    a = ap.parse_args()
    if a.analyse:
        analyse(a)
    else:
        run(a)


if __name__ == "__main__":
    main()
