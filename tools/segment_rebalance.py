"""Frame-to-frame segment starts for the K-segment traversal (tools/segment_model.c, skip form).

A GPU launch cannot know a ray's iteration quantiles before tracing it.  What it can keep is the
previous frame's starts and, per segment, the iterations it spent after arming (its share of the
continuous trace, c_k).  The next frame's starts put the cumulative shares at j/K of the total by
interpolating linearly in t between the old starts (the ray entry at 0, the end t -- hit or cube
exit -- at the total).  This script runs that rule over a sequence of frames and prints, per frame:
mismatches against the continuous oracle, the heaviest tile chain in the two wave layouts
(segment-major: wave k = segment k of 64 rays; ray-major: a wave = 64 / K rays x K segments, the
lanes of a ray adjacent), and the heavy tiles' wave trips against the continuous tile waves.

  python tools/segment_rebalance.py gpurun_out/r04i/c3_pool.npz --k 4 --frames 5 [--moving] [--init cube|quantile]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from oracle import oracle as orc  # noqa: E402
from raytracingtest_amd.camera import main_light  # noqa: E402
import segment_model as sm  # noqa: E402


def rebalance(bounds, seg, armed, status, fin, tent, texit, K):
    """New starts (n, K-1) from one frame's segments."""
    n = len(bounds)
    final = np.argmax(status != 2, axis=1)                      # the first segment that did not stop
    c = seg.astype(np.float64) - armed.astype(np.float64)       # continuous iterations after arming
    ks = np.arange(K)[None, :]
    c = np.where(ks <= final[:, None], c, 0.0)
    t_end = np.where(np.isfinite(fin["t"]), fin["t"].astype(np.float64) / 2048.0, texit.astype(np.float64))
    tp = np.concatenate([tent[:, None].astype(np.float64), bounds.astype(np.float64), t_end[:, None]], axis=1)
    cum = np.concatenate([np.zeros((n, 1)), np.cumsum(c, axis=1)], axis=1)     # at t_0 .. t_K
    # points beyond the final segment carry no information: collapse them onto the end
    tp[:, 1:K] = np.where(ks[:, 1:] <= final[:, None], tp[:, 1:K], t_end[:, None])
    tp[:, K] = t_end
    tot = cum[:, K]
    out = np.array(bounds, np.float64)
    for j in range(1, K):
        target = tot * j / K
        # segment holding the target: first k with cum[k+1] >= target
        k = np.argmax(cum[:, 1:] >= target[:, None] - 1e-9, axis=1)
        c0, c1 = cum[np.arange(n), k], cum[np.arange(n), k + 1]
        t0, t1 = tp[np.arange(n), k], tp[np.arange(n), k + 1]
        f = np.where(c1 > c0, (target - c0) / np.maximum(c1 - c0, 1e-9), 0.0)
        out[:, j - 1] = np.where(tot > 0, t0 + f * (t1 - t0), bounds[:, j - 1])
    return np.ascontiguousarray(np.maximum.accumulate(out, axis=1), np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--moving", action="store_true", help="pan one step per frame instead of holding the view")
    ap.add_argument("--init", default="cube", choices=["cube", "quantile"])
    ap.add_argument("--mode", default="hlsl")
    ap.add_argument("--frac", type=float, default=0.5)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    a = ap.parse_args()
    W, H, K = 1920, 1080, a.k
    z = np.load(a.npz)
    svo = orc.OracleSVO(nodes=z["nodes"], attachments=z["attachments"])
    L = sm.lib()
    mode = orc.STACK_HLSL if a.mode == "hlsl" else orc.STACK_EXACT
    light = main_light()

    def ocam(step):
        c2w, ip = sm.pan_camera(step).uniforms(W, H)
        return orc.make_camera(c2w, ip, (0.5, 0.5), light)

    n = W * H
    bounds = None
    for f in range(a.frames):
        cam = ocam(1 + f if a.moving else 1)
        h = sm.hints(L, svo, cam, W, H, mode, K, a.threads)
        if bounds is None:
            if a.init == "quantile":   # the previous frame traced continuously
                bounds = np.ascontiguousarray(sm.hints(L, svo, ocam(0 if a.moving else 1), W, H, mode, K, a.threads)["q"])
            else:
                fk = (np.arange(1, K, dtype=np.float32) / np.float32(K))[None, :]
                bounds = np.ascontiguousarray(h["tent"][:, None] + (h["texit"] - h["tent"])[:, None] * fk, np.float32)
        bounds = np.ascontiguousarray(np.maximum.accumulate(bounds, axis=1), np.float32)
        fin = np.zeros(n, orc.HIT_DTYPE)
        seg = np.zeros((n, K), np.uint32)
        it2 = np.zeros(n, np.uint32)
        mism = np.zeros(n, np.uint8)
        skips = np.zeros(n, np.uint32)
        armed = np.zeros((n, K), np.uint32)
        status = np.zeros((n, K), np.uint8)
        L.segm_run(ctypes.byref(svo.s), ctypes.byref(cam), W, H, mode, K, bounds.ctypes.data, 16, 1, a.threads,
                   fin.ctypes.data, seg.ctypes.data, it2.ctypes.data, mism.ctypes.data, skips.ctypes.data,
                   armed.ctypes.data, status.ctypes.data)
        cont = sm.tiles_of(h["it"].reshape(H, W).astype(np.int64), W, H).max(1)
        M = int(cont.max())
        heavy = cont >= a.frac * M
        st = sm.tiles_of(seg.reshape(H, W, K).astype(np.int64), W, H)          # tiles x 64 x K
        seg_major = st.max(1)                                                 # tiles x K waves
        ray_major = st.reshape(len(st), K, 64 // K, K).max(axis=(2, 3))        # tiles x K waves (rows)
        top = np.argsort(-cont)[:6]
        print(f"frame {f}: mismatches {int(mism.sum())} | continuous top {[int(cont[t]) for t in top]}"
              f" | segment-major {[int(seg_major[t].max()) for t in top]}, heavy wave trips"
              f" {int(cont[heavy].sum())} -> {int(seg_major[heavy].sum())}"
              f" | ray-major {[int(ray_major[t].max()) for t in top]}, {int(ray_major[heavy].sum())}"
              f" | heavy max: seg {int(seg_major[heavy].max())} ray {int(ray_major[heavy].max())}", flush=True)
        bounds = rebalance(bounds, seg, armed, status, fin, h["tent"], h["texit"], K)


if __name__ == "__main__":
    main()
