"""Model of beam starts (MODEL ONLY -- tools/segment_model.c, nothing in the product
loads it).  Every ray of the C3 frame against the CPU oracle (oracle/svo_oracle.c):

  cone     the ideal per-tile bound: a best-first search over the octree for the nearest box the
           cone around the tile's 64 rays touches (segm_beam), terminal at a leaf or at the cut
           scale -- what a start at that bound saves, before any cost of finding it;
  splat    the kernel's own rule (svo_kernel.hip beam_splat_kernel, restated in numpy): the nodes at
           the splat depth projected onto the screen, each tile's bound the minimum distance of the
           boxes whose projection (corner hull, clipped at the camera plane) touches the tile's
           pixel area; checked against every hit ray's oracle t (bound <= t, pixel offsets 0, 0.5 and
           1) and traced from it (segm_beam_run: the exact skip form, armed at the first event past
           the start; records compared with the continuous walk's).

  python tools/beam_model.py gpurun_out/r04i/c3_pool.npz --cameras flyover,main --cuts 13,15,17
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import segment_model as sm  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from raytracingtest_amd.camera import CAMERAS, main_light  # noqa: E402

f32 = np.float32


def bind(L):
    vp, i = ctypes.c_void_p, ctypes.c_int
    L.segm_beam.argtypes = [vp, vp, i, i, i, i, i, vp, vp, i, i]
    L.segm_beam_run.argtypes = [vp, vp, i, i, i, vp, i, vp, vp, vp]
    return L


def boxes_at(nodes, depth, leaves=False):
    """Lower corners (SVO space) of the non-leaf nodes at `depth` (svo_rt.hip build_beam_boxes; this
    pool has its leaves at the deepest level only); leaves=True: every valid child at the last level
    (the voxels themselves when depth is the pool's, beam_back 0)."""
    lo = (nodes & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    first = (nodes >> np.uint64(32)).astype(np.uint32)
    pc = np.array([bin(v).count("1") for v in range(256)])
    cur, pos, size = np.array([0]), np.zeros((1, 3)), 1.0
    for d in range(depth):
        m, v = lo[cur] & 0xFF, (lo[cur] >> 8) & 0xFF
        nxt, npos = [], []
        half = size / 2
        for c in range(8):   # bit c of the masks: upper half on axis k iff bit k of c
            inner = ((m >> c) & 1).astype(bool) & ((v >> c) & 1).astype(bool)
            if leaves and d == depth - 1:   # the last level: every valid child, leaf or not
                inner = ((v >> c) & 1).astype(bool)
            ptr = first[cur].astype(np.int64) + pc[m & ((1 << c) - 1)]
            nxt.append(ptr[inner])
            npos.append(pos[inner] + np.array([c & 1, (c >> 1) & 1, (c >> 2) & 1]) * half)
        cur, pos, size = np.concatenate(nxt), np.concatenate(npos), half
    return pos + 1.0, size


def splat(cam, P, size, W, H, cell=8):
    """The kernel's per-tile bounds (tile, 64x64 super tile, global), as a per-pixel image; `cell`:
    the finest cell's size in pixels (the kernel's 8; smaller: what finer cells would give)."""
    c2w = np.array(cam.c2w[:], f32)
    ip = np.array(cam.inv_proj[:], f32)
    A, B, C = (np.array([sum(float(c2w[k * 4 + r]) * float(ip[col * 4 + k]) for k in range(3)) for r in range(3)])
               for col in (0, 1, 3))
    M = np.stack([2 * A / W, 2 * B / H, C - A - B], 1)
    Minv = np.linalg.inv(M).astype(f32)
    D = [M @ np.array([fx, fy, 1.0]) for fx, fy in ((-1, -1), (W + 1, -1), (W + 1, H + 1), (-1, H + 1))]
    mid = M @ np.array([W / 2, H / 2, 1.0])
    planes = []
    for j in range(4):
        n = np.cross(D[j], D[(j + 1) % 4])
        n = n * (1 if n @ mid > 0 else -1)
        planes.append((n / np.linalg.norm(n)).astype(f32))
    org = (c2w[12:15] * f32(1 / 32) + f32(1.5)).astype(f32)
    lo = P.astype(f32)
    sz = np.broadcast_to(np.asarray(size, f32), (len(P),)).astype(f32)   # per box (a mixed list) or one
    rel = lo - org
    m = np.maximum(np.maximum(rel, -(rel + sz[:, None])), 0)
    dist = np.sqrt((m * m).sum(1)).astype(f32)
    span = np.abs(rel).sum(1) + 3 * sz
    keep = np.ones(len(P), bool)
    for n in planes:
        keep &= ~((rel @ n + sz * np.maximum(n, 0).sum()) < -1e-5 * span)
    q0 = rel @ Minv.T
    g = Minv.T   # row k: the step along axis k in q
    q = np.stack([q0 + sz[:, None] * ((c & 1) * g[0] + ((c >> 1) & 1) * g[1] + ((c >> 2) & 1) * g[2])
                  for c in range(8)], 1)
    qz = q[..., 2]
    zmax = qz.max(1)
    keep &= zmax > 0
    glob = keep & (dist <= 1e-3 * sz)
    eps = zmax * 1e-5
    x0 = np.full(len(P), np.inf, f32)
    x1, y0, y1 = -x0.copy(), x0.copy(), -x0.copy()
    with np.errstate(all="ignore"):
        for c in range(8):
            ok = qz[:, c] > eps
            fx, fy = q[:, c, 0] / qz[:, c], q[:, c, 1] / qz[:, c]
            x0, x1 = np.where(ok, np.minimum(x0, fx), x0), np.where(ok, np.maximum(x1, fx), x1)
            y0, y1 = np.where(ok, np.minimum(y0, fy), y0), np.where(ok, np.maximum(y1, fy), y1)
            for bit in (1, 2, 4):
                if c & bit:
                    continue
                d = c | bit
                cross = (qz[:, c] > eps) != (qz[:, d] > eps)
                s = (eps - qz[:, c]) / (qz[:, d] - qz[:, c])
                fx = (q[:, c, 0] + s * (q[:, d, 0] - q[:, c, 0])) / eps
                fy = (q[:, c, 1] + s * (q[:, d, 1] - q[:, c, 1])) / eps
                x0, x1 = np.where(cross, np.minimum(x0, fx), x0), np.where(cross, np.maximum(x1, fx), x1)
                y0, y1 = np.where(cross, np.minimum(y0, fy), y0), np.where(cross, np.maximum(y1, fy), y1)
    x0, y0, x1, y1 = x0 - 0.05, y0 - 0.05, x1 + 0.05, y1 + 0.05
    keep &= (x1 >= 0) & (y1 >= 0) & (x0 <= W) & (y0 <= H)
    tx_, ty_, sx_, sy_ = (W + cell - 1) // cell, (H + cell - 1) // cell, (W + 63) // 64, (H + 63) // 64
    per = 64 // cell   # cells per super tile side
    tiles, sup, gl = np.full(tx_ * ty_, np.inf, f32), np.full(sx_ * sy_, np.inf, f32), np.inf
    if glob.any():
        gl = min(gl, float(dist[glob].min()))
    k = keep & ~glob
    with np.errstate(all="ignore"):
        tx0 = (np.maximum(x0, 0) / cell).astype(np.int64)
        ty0 = (np.maximum(y0, 0) / cell).astype(np.int64)
        tx1 = np.minimum((np.minimum(x1, W) / cell).astype(np.int64), tx_ - 1)
        ty1 = np.minimum((np.minimum(y1, H) / cell).astype(np.int64), ty_ - 1)
    nt = (tx1 - tx0 + 1) * (ty1 - ty0 + 1)
    for i in np.flatnonzero(k & (nt <= 32)):
        for ty in range(ty0[i], ty1[i] + 1):
            row = tiles[ty * tx_ + tx0[i]: ty * tx_ + tx1[i] + 1]
            np.minimum(row, dist[i], out=row)
    stats = {"boxes_in_view": int(keep.sum()), "tile_writes": int(nt[k & (nt <= 32)].sum()), "super": 0,
             "global": int(glob.sum())}
    for i in np.flatnonzero(k & (nt > 32)):
        sx0, sx1, sy0, sy1 = tx0[i] // per, tx1[i] // per, ty0[i] // per, ty1[i] // per
        if (sx1 - sx0 + 1) * (sy1 - sy0 + 1) <= 32:
            stats["super"] += 1
            for sy in range(sy0, sy1 + 1):
                row = sup[sy * sx_ + sx0: sy * sx_ + sx1 + 1]
                np.minimum(row, dist[i], out=row)
        else:
            stats["global"] += 1
            gl = min(gl, float(dist[i]))
    ys, xs = np.mgrid[0:H, 0:W]
    img = np.minimum(np.minimum(tiles[(ys // cell) * tx_ + (xs // cell)], sup[(ys >> 6) * sx_ + (xs >> 6)]), f32(gl))
    return img.astype(f32), stats


def kernel_start(cam, img, W, H, off):
    """beam_start(): bound (1 - 2^-16) - (2 sum |coef| + sum |bias|) 2^-20, -inf for an axis-parallel ray."""
    c2w, ip = np.array(cam.c2w[:], np.float64), np.array(cam.inv_proj[:], np.float64)
    u = (np.arange(W)[None, :] + off[0]) / W * 2 - 1
    v = (np.arange(H)[:, None] + off[1]) / H * 2 - 1
    pd = [ip[0 * 4 + r] * u + ip[1 * 4 + r] * v + ip[3 * 4 + r] for r in range(3)]
    dr = [sum(c2w[k * 4 + r] * pd[k] for k in range(3)) for r in range(3)]
    nrm = np.sqrt(dr[0] ** 2 + dr[1] ** 2 + dr[2] ** 2)
    o3 = c2w[12:15] / 32 + 1.5
    with np.errstate(all="ignore"):
        coef = [1 / np.abs(dr[r] / nrm) for r in range(3)]
        zero = (np.abs(dr[0]) < 1e-9) | (np.abs(dr[1]) < 1e-9) | (np.abs(dr[2]) < 1e-9)
        mg = (2 * (coef[0] + coef[1] + coef[2]) + sum(coef[r] * (np.abs(o3[r]) + 3) for r in range(3))) * 2.0 ** -20
        s = img * f32(1 - 2 ** -16) - mg
    s = np.where(np.isnan(s) | zero, -np.inf, s)
    return np.ascontiguousarray(s.astype(f32).reshape(-1)), zero


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--cameras", default="flyover,main")
    ap.add_argument("--cuts", default="13,15,17", help="cone model: terminal scales (13 = the leaves of C3)")
    ap.add_argument("--splat-depth", type=int, default=8)
    ap.add_argument("--leaves", action="store_true", help="the splat's last level takes every valid child (voxels)")
    ap.add_argument("--cells", default="8", help="comma list of finest-cell sizes in pixels (the kernel: 8)")
    ap.add_argument("--offsets", default="0.5,0,1", help="pixel offsets checked (the first also traced)")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    a = ap.parse_args()
    W, H = 1920, 1080
    z = np.load(a.npz)
    svo = orc.OracleSVO(nodes=z["nodes"], attachments=z["attachments"])
    L = bind(sm.lib())
    P, size = boxes_at(z["nodes"].astype(np.uint64), a.splat_depth, a.leaves)
    print(f"C3 pool {len(z['nodes'])} nodes; splat depth {a.splat_depth}: {len(P)} boxes", flush=True)
    for name in a.cameras.split(","):
        c2w, ipm = (sm.pan_camera(1) if name == "flyover" else CAMERAS[name]()).uniforms(W, H)
        cam = orc.make_camera(c2w, ipm, (0.5, 0.5), main_light())
        n = W * H
        itc, itb, mism = np.zeros(n, np.uint32), np.zeros(n, np.uint32), np.zeros(n, np.uint8)

        def run(start):
            L.segm_beam_run(ctypes.byref(svo.s), ctypes.byref(cam), W, H, orc.STACK_HLSL, start.ctypes.data,
                            a.threads, itc.ctypes.data, itb.ctypes.data, mism.ctypes.data)
            cont = sm.tiles_of(itc.reshape(H, W).astype(np.int64), W, H)
            bb = sm.tiles_of(itb.reshape(H, W).astype(np.int64), W, H)
            return (f"mismatches {int(mism.sum())}; ray trips {cont.sum() / 1e6:.2f}M -> {bb.sum() / 1e6:.2f}M "
                    f"({bb.sum() / cont.sum():.3f}); wave trips {int(cont.max(1).sum())} -> {int(bb.max(1).sum())} "
                    f"({bb.max(1).sum() / cont.max(1).sum():.3f}); heaviest wave {int(cont.max())} -> {int(bb.max())}")

        for cut in (int(c) for c in a.cuts.split(",") if c):
            ty, tx = H // 8, W // 8
            tb, pops = np.zeros(ty * tx, f32), np.zeros(ty * tx, np.uint32)
            L.segm_beam(ctypes.byref(svo.s), ctypes.byref(cam), W, H, 8, cut, a.threads, tb.ctypes.data,
                        pops.ctypes.data, 0, 0)
            img = np.full((H, W), -np.inf, f32)
            img[:ty * 8, :tx * 8] = np.repeat(np.repeat(tb.reshape(ty, tx), 8, 0), 8, 1)
            start = np.ascontiguousarray(np.where(np.isfinite(img), img * f32(1 - 2 ** -14), img).reshape(-1))
            print(f"{name} cone, terminal scale {cut}: search pops/tile mean {pops.mean():.1f} max {pops.max()}; "
                  + run(start), flush=True)
        offs = [(float(o), float(o)) for o in a.offsets.split(",")]
        for cell, off in ((int(c), o) for c in a.cells.split(",") for o in offs):
            cam = orc.make_camera(c2w, ipm, off, main_light())
            img, st = splat(cam, P, size, W, H, cell)
            hits, _, _ = orc.render(svo, cam, W, H, orc.STACK_HLSL, want_rgba=False, want_fetches=False)
            start, zero = kernel_start(cam, img, W, H, off)
            th = (hits["t"] / f32(2048)).reshape(H, W)
            hit = ((hits["flags"] & 1).reshape(H, W) != 0) & ~zero
            bad = int(np.count_nonzero(hit & (start.reshape(H, W) > th)))
            print(f"{name} splat, cell {cell}, offset {off}: {st}; hit rays {int(hit.sum())}, start > oracle t for {bad}"
                  + ("; " + run(start) if off == offs[0] else ""), flush=True)


if __name__ == "__main__":
    main()
