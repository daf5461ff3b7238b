"""A/B of the segmented heavy tiles on the C3 frame: render-kernel time of the
whole 1920x1080 flyover frame (N = 1) and of rank 1's round-robin 8-row band at N = 2, 4, 8 (the
strong split's per-GPU launch), with segments off and on (and the latency form's automatic choice
in both), interleaved in one process; each variant is an svo_config (include/svo_rt.h) given to
the context it creates.  Library
events, median of --timed launches after a warmup past the clock ramp.

  python tools/seg_ab.py [--camera flyover] [--rounds 2] > gpurun_out/seg_ab.json
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
    ap.add_argument("--camera", default="flyover")
    ap.add_argument("--timed", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variants", default="off,auto",
                    help="comma list of: off (segments = 0), auto (the library's defaults), or '+'-joined "
                         "l<hex> (seg_table_latency: K per cost class, class 0 in the low nibble), i<hex> "
                         "(seg_table_issue), t<hex> (seg_table_thin), nobeam (beam = 0) and norelayout (relayout = 0)")
    ap.add_argument("--cap", default=None, help="seg_cap")
    ap.add_argument("--cameras", default=None, help="comma list (default: --camera)")
    a = ap.parse_args()
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = CONFIGS["C3"]
    W, H = cfg["width"], cfg["height"]
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"], device=0)
    hits = torch.empty(W * H * 24, dtype=torch.uint8, device="cuda")
    rgba = torch.empty(W * H * 16, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    out = {"frame": f"{W}x{H}", "rows": []}
    cams = (a.cameras or a.camera).split(",")
    for rnd in range(a.rounds):
        for name in a.variants.split(","):
            conf = {}
            for part in name.split("+"):
                if part == "off":
                    conf["segments"] = 0
                elif part.startswith("l"):     # l<hex>: the class table of latency-bound launches
                    conf["seg_table_latency"] = int(part[1:], 16)
                elif part.startswith("i"):     # i<hex>: the same for issue-bound launches
                    conf["seg_table_issue"] = int(part[1:], 16)
                elif part.startswith("t"):     # t<hex>: the table of thin latency-bound launches
                    conf["seg_table_thin"] = int(part[1:], 16)
                elif part == "nobeam":         # rays from the cube entry
                    conf["beam"] = 0
                elif part == "norelayout":     # keep the first order built at a new class table
                    conf["relayout"] = 0
            if a.cap:
                conf["seg_cap"] = int(a.cap, 0)
            for cam in cams:
                rm = RaytracingMaster(device=0, capacity_nodes=len(svo), config=conf)
                rm.SetSVOBuffer(svo)
                rm.UpdateShaderParameters(CAMERAS[cam](), W, H)
                for _ in range(400):   # past the DVFS ramp
                    rm.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), stream=s.cuda_stream)
                torch.cuda.synchronize()
                for N in (1, 2, 4, 8):
                    band = None if N == 1 else (8, 1, N)
                    for _ in range(40):
                        rm.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), band=band, stream=s.cuda_stream)
                    rm.set_kernel_timing(True)
                    rm.kernel_time()
                    for _ in range(a.timed):
                        rm.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), band=band, stream=s.cuda_stream)
                    t = rm.stage_times()
                    rm.set_kernel_timing(False)
                    row = {"round": rnd, "variant": name, "camera": cam, "N": N,
                           "kernel_ms_median": round(float(np.median(t)), 4),
                           "kernel_ms_p10": round(float(np.percentile(t, 10)), 4)}
                    out["rows"].append(row)
                    print(json.dumps(row), file=sys.stderr, flush=True)
                rm.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
