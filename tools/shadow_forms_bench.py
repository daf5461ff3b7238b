"""Experiment: the three forms of C3's '+1 shadow ray' pass on one MI355X
(DESIGN.md 3.2): fused into the primary launch (default), a second launch over
the 8x8 tiles (SVO_FUSED_SHADOWS=0), and a second launch over the compacted hit
list (SVO_SHADOW_COMPACT=1).  Time = HIP events around the whole render
(primary + shadow kernels + the compaction), mean over --steps frames after
warmup; every form's hit records are compared with the fused form's.

  python tools/shadow_forms_bench.py [--steps 40] [--cameras flyover main]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FORMS = {"fused": {}, "two_pass_tiles": {"SVO_FUSED_SHADOWS": "0"}, "compacted_list": {"SVO_SHADOW_COMPACT": "1"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--cameras", nargs="+", default=["flyover", "main"])
    a = ap.parse_args()
    import torch
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    svo = build_sampler_svo(4, 11, device=0)
    W, H = 1920, 1080
    s = torch.cuda.Stream()
    hits = torch.empty(W * H * 24, dtype=torch.uint8, device="cuda")
    rgba = torch.empty(W * H * 4, dtype=torch.float32, device="cuda")

    def run(cam, env, shadows):
        for k in ("SVO_FUSED_SHADOWS", "SVO_SHADOW_COMPACT"):
            os.environ.pop(k, None)
        os.environ.update(env)
        rm = RaytracingMaster(device=0, capacity_nodes=len(svo))   # the switches are read here
        rm.SetSVOBuffer(svo)
        rm.UpdateShaderParameters(CAMERAS[cam](), W, H)
        rm.SetShadowRays(shadows)
        for _ in range(8):
            rm.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), stream=s.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.steps):
            rm.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), stream=s.cuda_stream)
        e1.record(s)
        e1.synchronize()
        rm.close()
        return e0.elapsed_time(e1) / a.steps, hits.clone()

    for cam in a.cameras:
        prim, _ = run(cam, {}, False)
        print(f"{cam}: primary rays only {prim:.4f} ms/frame", flush=True)
        ref = None
        for name, env in FORMS.items():
            ms, h = run(cam, env, True)
            if ref is None:
                ref = h
            n_hit = int((h.view(-1, 24)[:, 6] & 1).sum().item())
            print(f"  {name}: {ms:.4f} ms/frame (shadow part {ms - prim:.4f} ms, {n_hit} hits); "
                  f"records identical to fused: {bool(torch.equal(h, ref))}", flush=True)


if __name__ == "__main__":
    main()
