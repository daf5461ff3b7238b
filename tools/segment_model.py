"""Model of tracing one primary ray as K t-segments (tools/segment_model.c).

Per frame and stack mode, with the segment starts t_1..t_{K-1} chosen by
  cube      uniform over [t_entry, cube exit];
  hint      uniform over [t_entry, t_end], t_end = the hint frame's hit t (cube exit on a miss);
  quantile  the hint frame's t_min at iterations k n / K (n = its iteration count),
and the hint frame either this frame (`held`: a held view) or, for the flyover camera, the frame
one pan step earlier (`moving`: tools/moving_camera.py's 2 mrad orbit), it reports
  * rays whose combined record differs from the continuous oracle's (parent, hit_idx, scale, t bits);
  * the heaviest chain: per 8x8 tile, segment-major waves (wave k = segment k of the tile's 64 rays),
    the tile's chain = its longest segment wave, against the continuous tile wave;
  * the same for rank 1's band of an N-way 8-row round-robin split;
  * wave trips summed over the tiles that would be segmented (cost >= FRAC x the frame's heaviest).

  python tools/segment_model.py gpurun_out/r04i/c3_pool.npz --camera flyover --k 2 4 8
"""
import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as orc  # noqa: E402
from raytracingtest_amd.camera import CAMERAS, FLYOVER_EYE, FLYOVER_TARGET, main_light, overview_camera  # noqa: E402

LIB = os.path.join(ROOT, "tools", "build", "libsegmodel.so")


def lib():
    src = os.path.join(ROOT, "tools", "segment_model.c")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-pthread",
                        "-shared", "-o", LIB, src, os.path.join(ROOT, "oracle", "svo_oracle.c"), "-lm"], check=True)
    L = ctypes.CDLL(LIB)
    vp, i = ctypes.c_void_p, ctypes.c_int
    L.segm_hints.argtypes = [vp, vp, i, i, i, i, i, vp, vp, vp, vp, vp]
    L.segm_run.argtypes = [vp, vp, i, i, i, i, vp, i, i, i, vp, vp, vp, vp, vp, vp, vp]
    return L


def tiles_of(a, W, H):
    """(H, W, ...) -> (tiles, 64, ...), tiles row-major, lanes row-major in the tile."""
    tx, ty = W // 8, H // 8
    rest = a.shape[2:]
    b = a[:ty * 8, :tx * 8].reshape((ty, 8, tx, 8) + rest)
    b = np.moveaxis(b, 2, 1)
    return b.reshape((ty * tx, 64) + rest)


def pan_camera(step):
    """tools/moving_camera.py's orbit of the flyover eye, `step` frames in."""
    ang = 0.002 * step
    ex, ey, ez = FLYOVER_EYE
    eye = (ex + 0.5 * np.sin(ang), ey, ez + 0.5 * (1.0 - np.cos(ang)))
    return overview_camera(eye, FLYOVER_TARGET)


def hints(L, svo, cam, W, H, mode, K, threads):
    n = W * H
    q = np.zeros((n, max(K - 1, 1)), np.float32)
    tend, tent, texit = (np.zeros(n, np.float32) for _ in range(3))
    it = np.zeros(n, np.uint32)
    L.segm_hints(ctypes.byref(svo.s), ctypes.byref(cam), W, H, mode, K, threads,
                 q.ctypes.data, tend.ctypes.data, tent.ctypes.data, texit.ctypes.data, it.ctypes.data)
    return dict(q=q[:, :K - 1], tend=tend, tent=tent, texit=texit, it=it)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--camera", default="flyover")
    ap.add_argument("--k", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--modes", default="hlsl,exact")
    ap.add_argument("--frac", type=float, default=0.5, help="segment tiles with cost >= frac x heaviest")
    ap.add_argument("--band", type=int, default=8, help="report rank 1's band of an N-way 8-row split")
    ap.add_argument("--margin", type=int, default=16, help="ulps the stop lies past the next start")
    ap.add_argument("--form", default="skip", choices=["skip", "descent"],
                    help="skip: walk from the cube entry, skipping subtrees wholly before t_k (exact state); "
                         "descent: descend straight to t_k (margin rule)")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    a = ap.parse_args()
    W, H = a.width, a.height
    z = np.load(a.npz)
    svo = orc.OracleSVO(nodes=z["nodes"], attachments=z["attachments"])
    L = lib()
    light = main_light()
    if a.camera == "flyover":   # the frame is pan step 1; its hint frame this view or pan step 0
        cams = {"held": pan_camera(1), "moving": pan_camera(0)}
    else:
        cams = {"held": CAMERAS[a.camera]()}

    def ocam(c):
        c2w, ip = c.uniforms(W, H)
        return orc.make_camera(c2w, ip, (0.5, 0.5), light)

    cam = ocam(cams["held"])
    n_px = W * H
    ty, tx = H // 8, W // 8
    band_tiles = (np.arange(ty * tx) // tx) % a.band == 1
    print(f"frame {W}x{H}, camera {a.camera}, pool {len(z['nodes'])} nodes", flush=True)
    for mode_name in a.modes.split(","):
        mode = orc.STACK_HLSL if mode_name == "hlsl" else orc.STACK_EXACT
        for K in a.k:
            hs = {name: hints(L, svo, ocam(c), W, H, mode, K, a.threads) for name, c in cams.items()}
            now = hs["held"]
            cont_chain = tiles_of(now["it"].reshape(H, W).astype(np.int64), W, H).max(1)
            M = int(cont_chain.max())
            heavy = cont_chain >= a.frac * M
            fk = (np.arange(1, K, dtype=np.float32) / np.float32(K))[None, :]
            runs = [("held", "cube", now["tent"][:, None] + (now["texit"] - now["tent"])[:, None] * fk)]
            for name, h in hs.items():
                runs.append((name, "hint", h["tent"][:, None] + (h["tend"] - h["tent"])[:, None] * fk))
                runs.append((name, "quantile", h["q"]))
            for hname, sname, bounds in runs:
                bounds = np.ascontiguousarray(np.maximum.accumulate(bounds, axis=1), np.float32)
                fin = np.zeros(n_px, orc.HIT_DTYPE)
                seg = np.zeros((n_px, K), np.uint32)
                it2 = np.zeros(n_px, np.uint32)
                mism = np.zeros(n_px, np.uint8)
                skips = np.zeros(n_px, np.uint32)
                L.segm_run(ctypes.byref(svo.s), ctypes.byref(cam), W, H, mode, K, bounds.ctypes.data, a.margin,
                           1 if a.form == "skip" else 0, a.threads,
                           fin.ctypes.data, seg.ctypes.data, it2.ctypes.data, mism.ctypes.data, skips.ctypes.data, None, None)
                assert (it2 == now["it"]).all()
                seg_chain = tiles_of(seg.reshape(H, W, K).astype(np.int64), W, H).max(1)   # tiles x K
                tile_chain = np.where(heavy, seg_chain.max(1), cont_chain)
                top = np.argsort(-cont_chain)[:6]
                tc, ts = int(cont_chain[heavy].sum()), int(seg_chain[heavy].sum())
                print(f"{mode_name:5s} K={K} {hname:6s} {sname:8s}: mismatches {int(mism.sum()):5d}"
                      f" | heaviest {M} -> {int(tile_chain.max()):3d} ({100.0 * tile_chain.max() / M:5.1f} %)"
                      f" | band {int(cont_chain[band_tiles].max())} -> {int(tile_chain[band_tiles].max())}"
                      f" | top {[int(cont_chain[t]) for t in top]} -> {[int(tile_chain[t]) for t in top]}"
                      f" | {int(heavy.sum())} heavy tiles, wave trips {tc} -> {ts} ({ts / max(tc, 1):.2f}x)", flush=True)


if __name__ == "__main__":
    main()
