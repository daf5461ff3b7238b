"""Host cost of an upload (SetSVOBuffer: validation walk, the splat lists, the device copies) with and
without the held view's voxel list (svo_config.beam_back_held 0 against -1), per config.

  python tools/upload_cost.py [--configs C3,C5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C3,C5")
    a = ap.parse_args()
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.native_builder import build_sampler_svo
    for name in a.configs.split(","):
        cfg = CONFIGS[name]
        svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
        out = {"config": name, "nodes": len(svo)}
        for held in (-1, 0, -1, 0):
            m = RaytracingMaster(capacity_nodes=len(svo), config={"beam_back_held": held})
            t = time.perf_counter()
            m.SetSVOBuffer(svo)
            out.setdefault(f"upload_s_held{held}", []).append(round(time.perf_counter() - t, 3))
            m.close()
        print(json.dumps(out), flush=True)
        del svo


if __name__ == "__main__":
    main()
