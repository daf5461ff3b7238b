"""One-sample route against the render launch on the C3 frame: GPU span per
launch of render_frame (hits + RGBA32F, hits only) and of svo_render_samples with one sample per
launch -- a new jittered offset each launch, without the display words, and one fixed offset --
then render_frame again, per camera; optional svo_config fields as field=value after the cameras
(e.g. seg_jitter=1 seg_move=1).

  python tools/one_sample_ab.py flyover,overview [seg_jitter=1] > gpurun_out/one_sample.txt
"""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from bench import CONFIGS
from raytracingtest_amd import RaytracingMaster
from raytracingtest_amd.camera import CAMERAS, jitter_offsets
from raytracingtest_amd.native_builder import build_sampler_svo
cfg = CONFIGS["C3"]; W, H = cfg["width"], cfg["height"]
svo = build_sampler_svo(cfg["sampler"], cfg["max_level"], device=0)
hits = torch.empty(W * H * 24, dtype=torch.uint8, device="cuda")
rgba = torch.empty(W * H * 16, dtype=torch.uint8, device="cuda")
acc = torch.zeros(W * H * 4, dtype=torch.float32, device="cuda")
f8 = torch.empty(W * H, dtype=torch.int32, device="cuda")
s = torch.cuda.Stream(); offs = jitter_offsets(4096)
def span(fn, k=300):
    for _ in range(100): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(k): fn()
    e1.record(s); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k
CONF = {kv.split("=")[0]: int(kv.split("=")[1], 0) for kv in sys.argv[2:]}
for cam in sys.argv[1].split(","):
    rm = RaytracingMaster(device=0, capacity_nodes=len(svo), config=CONF); rm.SetSVOBuffer(svo)
    rm.UpdateShaderParameters(CAMERAS[cam](), W, H)
    n = [0]
    def r(): rm.render_frame(W, H, hits=hits.data_ptr(), rgba=rgba.data_ptr(), stream=s.cuda_stream)
    def rh(): rm.render_frame(W, H, hits=hits.data_ptr(), stream=s.cuda_stream)
    def s1():
        rm.render_samples(W, H, offs[np.arange(n[0], n[0] + 1) % len(offs)], n[0], acc.data_ptr(), rgba8=f8.data_ptr(), stream=s.cuda_stream); n[0] += 1
    def s1n():
        rm.render_samples(W, H, offs[np.arange(n[0], n[0] + 1) % len(offs)], n[0], acc.data_ptr(), stream=s.cuda_stream); n[0] += 1
    def s1fixed():
        rm.render_samples(W, H, offs[:1], n[0], acc.data_ptr(), rgba8=f8.data_ptr(), stream=s.cuda_stream); n[0] += 1
    print(json.dumps({"cam": cam, "render": span(r), "render_hits_only": span(rh), "s1": span(s1), "s1_no_rgba8": span(s1n),
                      "s1_fixed_offset": span(s1fixed), "render_again": span(r)}), flush=True)
    rm.close()
