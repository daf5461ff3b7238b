"""The drop-in's frame loop on its own (bench.py dropin_loop_rates: held view with a fixed offset,
jittered, and a pan with a new view every frame), for A/Bs of the moving-camera and jitter policy
without the whole bench.  Prints one JSON line per pose.

  python tools/dropin_loop.py [--config C3] [--poses flyover,main] [--frames 300] [--set key=value ...]

--set applies svo_config fields (include/svo_rt.h) to the context before the measurement.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--poses", default="flyover,main")
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--set", action="append", default=[], help="svo_config field=value")
    a = ap.parse_args()
    import torch
    import bench
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = bench.CONFIGS[a.config]
    W, H = cfg["width"], cfg["height"]
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    rm = RaytracingMaster(capacity_nodes=len(svo))
    rm.SetSVOBuffer(svo)
    if a.set and hasattr(rm, "set_config"):
        kv = {}
        for s in a.set:
            k, v = s.split("=", 1)
            kv[k] = float(v) if "." in v else int(v, 0)
        rm.set_config(**kv)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    for pose in a.poses.split(","):
        rm.UpdateShaderParameters(CAMERAS[pose](), W, H)
        h = torch.empty(W * H * 24, dtype=torch.uint8, device=dev)
        for _ in range(400):   # past the clock ramp
            rm.render_device(W, H, hits_ptr=h.data_ptr(), stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        args = argparse.Namespace(camera=pose, stack_mode=cfg["stack_mode"])
        dropin, pan = bench.dropin_loop_rates(rm, W, H, args, dev, stream, frames=a.frames)
        print(json.dumps({"pose": pose, "config": a.config, "set": a.set, "dropin_loop": dropin, "pan": pan}),
              flush=True)
    rm.close()


if __name__ == "__main__":
    main()
