"""Model (test infrastructure only): a moving camera's splat list mixing the depth-8 boxes (far) with the
voxels of the coarse boxes whose projection is at least THR pixels (near), against the coarse and the
voxel lists -- tools/beam_model.py's splat and trace on the dumped C3 pool.

  python tools/hybrid_splat_model.py   (reads gpurun_out/r04i/c3_pool.npz)
"""
import sys, os, numpy as np, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tools"))
import beam_model as bm
import segment_model as sm
from oracle import oracle as orc
from raytracingtest_amd.camera import CAMERAS, main_light
f32 = np.float32
W, H = 1920, 1080
z = np.load(os.path.join(ROOT, "gpurun_out", "r04i", "c3_pool.npz"))
svo = orc.OracleSVO(nodes=z["nodes"], attachments=z["attachments"])
L = bm.bind(sm.lib())
nodes = z["nodes"].astype(np.uint64)
P8, s8 = bm.boxes_at(nodes, 8)
P10, s10 = bm.boxes_at(nodes, 10, leaves=True)
# the coarse box of every voxel: integer cell at depth 8
c8 = np.floor((P8 - 1.0) * 256 + 0.5).astype(np.int64)
k8 = (c8[:, 0] << 20) | (c8[:, 1] << 10) | c8[:, 2]
c10 = np.floor((P10 - 1.0) * 256).astype(np.int64)
k10 = (c10[:, 0] << 20) | (c10[:, 1] << 10) | c10[:, 2]
order8 = np.argsort(k8)
print("boxes", len(P8), len(P10), flush=True)
for name in ("flyover", "main"):
    c2w, ipm = (sm.pan_camera(1) if name == "flyover" else CAMERAS[name]()).uniforms(W, H)
    cam = orc.make_camera(c2w, ipm, (0.5, 0.5), main_light())
    org = np.array(c2w, np.float64).reshape(-1)[12:15] / 32 + 1.5
    # coarse box pixel size ~ size / dist * focal
    ip = np.array(ipm, np.float64).reshape(-1)
    focal = H / 2 / abs(ip[5]) if abs(ip[5]) > 0 else 500.0
    cen = P8 + s8 / 2
    d = np.linalg.norm(cen - org, axis=1)
    px = s8 / np.maximum(d, 1e-6) * focal
    n = W * H
    itc, itb, mism = np.zeros(n, np.uint32), np.zeros(n, np.uint32), np.zeros(n, np.uint8)
    def run(start):
        L.segm_beam_run(ctypes.byref(svo.s), ctypes.byref(cam), W, H, orc.STACK_HLSL, start.ctypes.data, 8,
                        itc.ctypes.data, itb.ctypes.data, mism.ctypes.data)
        cont = sm.tiles_of(itc.reshape(H, W).astype(np.int64), W, H)
        bb = sm.tiles_of(itb.reshape(H, W).astype(np.int64), W, H)
        return f"mism {int(mism.sum())}; wave trips {bb.max(1).sum() / cont.max(1).sum():.3f}; ray trips {bb.sum() / cont.sum():.3f}"
    for label, thr in (("coarse", None), ("fine", -1), ("hybrid16", 16.0), ("hybrid8", 8.0), ("hybrid4", 4.0), ("hybrid2", 2.0)):
        if thr is None:
            P, S = P8, np.full(len(P8), s8, f32)
        elif thr < 0:
            P, S = P10, np.full(len(P10), s10, f32)
        else:
            big = px >= thr
            bigkeys = np.sort(k8[big])
            sel = np.isin(k10, bigkeys)
            P = np.concatenate([P8[~big], P10[sel]]); S = np.concatenate([np.full((~big).sum(), s8, f32), np.full(sel.sum(), s10, f32)])
        img, st = bm.splat(cam, P, S, W, H, 8)
        start, zero = bm.kernel_start(cam, img, W, H, (0.5, 0.5))
        print(name, label, "boxes", len(P), run(start), flush=True)
