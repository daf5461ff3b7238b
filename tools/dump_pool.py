"""Build a BASELINE config's node pool on the GPU with the native builder and
save it (V2 nodes + attachments) as an .npz, so CPU-side tools (the oracle's
iteration-kind model, tools/trip_model.py) can work on the exact bench pool
without a GPU.

  python tools/dump_pool.py [--config C3] [--out gpurun_out/c3_pool.npz]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--out", default="gpurun_out/c3_pool.npz")
    a = ap.parse_args()
    from bench import CONFIGS
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = CONFIGS[a.config]
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    np.savez_compressed(a.out, nodes=svo.to_v2(), attachments=svo.attachments, max_level=cfg["max_level"])
    print(f"{a.config}: {len(svo)} nodes -> {a.out} ({os.path.getsize(a.out) / 1e6:.1f} MB)")


if __name__ == "__main__":
    main()
