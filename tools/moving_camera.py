"""The interactive case: a camera that moves every frame (RaytracingMaster.cs:55-74 renders a
fresh view per frame).  C3 frame, flyover pose; per-frame wall time (host clock, K frames between
two synchronizes, no events in the timed frames) for a static view and for a slow pan (a new view
every frame, camera uniforms precomputed so the host stays ahead), then the render kernel's own
time in both (library events, a separate pass).  The difference is what a moving camera costs
beyond the kernel: the dispatch-order rebuild behind every launch at a new view.

  python tools/moving_camera.py [--frames 300]     (SVO_MOVE_EVERY=k: the library rebuilds the order every k-th moving frame)
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=300)
    ap.add_argument("--cycle", type=int, default=0,
                    help="diagnostics: cycle through the first k views of the pan (a new view per frame, "
                         "views repeating) instead of panning on")
    ap.add_argument("--move-every", type=int, default=None, help="svo_config.move_every (default: the library's)")
    a = ap.parse_args()
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster, _lib
    from raytracingtest_amd.camera import FLYOVER_EYE, FLYOVER_TARGET, main_light, overview_camera
    from raytracingtest_amd.raytracing_master import column_major
    cfg = CONFIGS["C3"]
    W, H = cfg["width"], cfg["height"]
    from raytracingtest_amd.native_builder import build_sampler_svo
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    rm = RaytracingMaster(capacity_nodes=len(svo), config={} if a.move_every is None else {"move_every": a.move_every})
    rm.SetSVOBuffer(svo)
    light = np.ascontiguousarray(main_light(), np.float32)
    views = []
    for i in range(a.frames + 1):
        ang = 0.002 * i   # a slow pan: the eye circles the flyover eye by 2 mrad per frame
        eye = (FLYOVER_EYE[0] + 3.0 * np.sin(ang), FLYOVER_EYE[1], FLYOVER_EYE[2] + 3.0 * (1.0 - np.cos(ang)))
        c2w, inv_proj = overview_camera(eye, FLYOVER_TARGET).uniforms(W, H)
        views.append((column_major(np.asarray(c2w, np.float32)), column_major(np.asarray(inv_proj, np.float32))))
    L = _lib.lib()

    def set_view(k):
        c, p = views[k]
        L.svo_set_camera(rm._ctx, c.ctypes.data, p.ctypes.data, 0.5, 0.5, light.ctypes.data)

    h = torch.empty(W * H * 24, dtype=torch.uint8, device="cuda")
    rg = torch.empty(W * H * 4, dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()

    def render():
        rm.render_device(W, H, hits_ptr=h.data_ptr(), rgba_ptr=rg.data_ptr(), stack_mode=0, stream=s.cuda_stream)

    set_view(0)
    torch.cuda.synchronize()
    for _ in range(400):   # past the clock ramp
        render()
    torch.cuda.synchronize()
    out = {}
    for rnd in range(2):
        for name in ("static", "moving"):
            set_view(0)
            render()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.frames):
                if name == "moving":
                    set_view(k % a.cycle + 1 if a.cycle else k + 1)
                render()
            t_host = time.perf_counter() - t0
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.frames * 1e3
            rm.set_kernel_timing(True)
            rm.kernel_time()
            for k in range(a.frames):
                if name == "moving":
                    set_view(k % a.cycle + 1 if a.cycle else k + 1)
                render()
            kms, n = rm.kernel_time()
            rm.set_kernel_timing(False)
            torch.cuda.synchronize()
            out.setdefault(name, []).append((ms, kms))
            print(f"move_every={a.move_every or 'default'} round {rnd} {name:6s}: {ms * 1e3:6.1f} us per frame (host issue {t_host / a.frames * 1e6:5.1f} us), "
                  f"render kernel {kms * 1e3:6.1f} us", flush=True)
    rm.close()


if __name__ == "__main__":
    main()
