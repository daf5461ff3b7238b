"""Independent first-hit checker: double-precision slab test of every leaf voxel.

Shares no code with the oracle's Laine-Karras traversal; used to pin the
traversal's hit voxel (up to ties) on the reference's `Text` SVO fixture."""
import numpy as np


def svo_space_ray(origin, direction):
    """NVIDIASVO.compute:15-19: o' = o / 32 + 1.5 (direction unchanged)."""
    o = np.asarray(origin, np.float64) / 32.0 + 1.5
    return o, np.asarray(direction, np.float64)


def first_hits(leaves, origins, dirs, chunk=64, min_overlap=1e-6):
    """leaves: rows (node, slot, L, ix, iy, iz).
    Returns (best_row, best_t, t_entry[rays, leaves], overlap[rays, leaves]).
    best_row / best_t consider only leaves the ray crosses over a length
    > min_overlap (edge/corner grazes are ties the float traversal may skip);
    t_entry is +inf for leaves the ray does not touch at all."""
    size = 2.0 ** -leaves[:, 2].astype(np.float64)
    lo = 1.0 + leaves[:, 3:6].astype(np.float64) * size[:, None]
    hi = lo + size[:, None]
    n = len(origins)
    best_row = np.full(n, -1, np.int64)
    best_t = np.full(n, np.inf)
    entries, overlaps = [], []
    for s in range(0, n, chunk):
        o = origins[s:s + chunk][:, None, :]
        d = dirs[s:s + chunk][:, None, :]
        with np.errstate(divide="ignore", invalid="ignore"):
            inv = 1.0 / d
            t0 = (lo[None] - o) * inv
            t1 = (hi[None] - o) * inv
        tmin = np.minimum(t0, t1)
        tmax = np.maximum(t0, t1)
        # zero direction component: inside the slab -> unbounded, outside -> miss
        par = (d == 0.0)
        inside = (o >= lo[None]) & (o <= hi[None])
        tmin = np.where(par, np.where(inside, -np.inf, np.inf), tmin)
        tmax = np.where(par, np.where(inside, np.inf, -np.inf), tmax)
        te = tmin.max(axis=2)
        tx = tmax.min(axis=2)
        hit = (te <= tx) & (tx >= 0.0)
        te = np.where(hit, np.maximum(te, 0.0), np.inf)
        ov = np.where(hit, tx - te, -np.inf)
        entries.append(te)
        overlaps.append(ov)
        solid = np.where(ov > min_overlap, te, np.inf)
        k = solid.argmin(axis=1)
        bt = solid[np.arange(len(solid)), k]
        best_row[s:s + chunk] = np.where(np.isfinite(bt), k, -1)
        best_t[s:s + chunk] = bt
    return best_row, best_t, np.concatenate(entries), np.concatenate(overlaps)


def first_hits_compact(leaves, origins, dirs, chunk=256, min_overlap=1e-6):
    """first_hits for whole frames: the same slab test, but per ray only
    (best_row, best_t, max_overlap) are kept (t_entry / overlap over all leaves
    would be rays x leaves doubles).  Runs on torch's CPU threads when torch
    is importable, else numpy."""
    try:
        import torch
        xp = "torch"
    except ImportError:   # pragma: no cover
        xp = "numpy"
    size = 2.0 ** -leaves[:, 2].astype(np.float64)
    lo = 1.0 + leaves[:, 3:6].astype(np.float64) * size[:, None]
    hi = lo + size[:, None]
    n = len(origins)
    best_row = np.full(n, -1, np.int64)
    best_t = np.full(n, np.inf)
    max_ov = np.full(n, -np.inf)
    if xp == "torch":
        tlo, thi = torch.from_numpy(lo)[None], torch.from_numpy(hi)[None]
    for s in range(0, n, chunk):
        o = np.asarray(origins[s:s + chunk], np.float64)[:, None, :]
        d = np.asarray(dirs[s:s + chunk], np.float64)[:, None, :]
        if xp == "torch":
            to, td = torch.from_numpy(o), torch.from_numpy(d)
            inv = 1.0 / td
            t0 = (tlo - to) * inv
            t1 = (thi - to) * inv
            tmin, tmax = torch.minimum(t0, t1), torch.maximum(t0, t1)
            par = td == 0.0
            inside = (to >= tlo) & (to <= thi)
            inf = torch.tensor(np.inf, dtype=torch.float64)
            tmin = torch.where(par, torch.where(inside, -inf, inf), tmin)
            tmax = torch.where(par, torch.where(inside, inf, -inf), tmax)
            te = tmin.amax(dim=2)
            tx = tmax.amin(dim=2)
            hit = (te <= tx) & (tx >= 0.0)
            te = torch.where(hit, te.clamp(min=0.0), inf)
            ov = torch.where(hit, tx - te, -inf)
            solid = torch.where(ov > min_overlap, te, inf)
            bt, k = solid.min(dim=1)
            bt, k, mo = bt.numpy(), k.numpy(), ov.amax(dim=1).numpy()
        else:
            with np.errstate(divide="ignore", invalid="ignore"):
                inv = 1.0 / d
                t0 = (lo[None] - o) * inv
                t1 = (hi[None] - o) * inv
            tmin, tmax = np.minimum(t0, t1), np.maximum(t0, t1)
            par = d == 0.0
            inside = (o >= lo[None]) & (o <= hi[None])
            tmin = np.where(par, np.where(inside, -np.inf, np.inf), tmin)
            tmax = np.where(par, np.where(inside, np.inf, -np.inf), tmax)
            te, tx = tmin.max(axis=2), tmax.min(axis=2)
            hit = (te <= tx) & (tx >= 0.0)
            te = np.where(hit, np.maximum(te, 0.0), np.inf)
            ov = np.where(hit, tx - te, -np.inf)
            solid = np.where(ov > min_overlap, te, np.inf)
            k = solid.argmin(axis=1)
            bt, mo = solid[np.arange(len(solid)), k], ov.max(axis=1)
        best_row[s:s + chunk] = np.where(np.isfinite(bt), k, -1)
        best_t[s:s + chunk] = bt
        max_ov[s:s + chunk] = mo
    return best_row, best_t, max_ov


def entry_exit(leaf, origin, direction, eps=2e-6):
    """(t_entry, t_exit) of one leaf box grown by eps per side (float-vs-double slack)."""
    size = 2.0 ** -float(leaf[2])
    lo = 1.0 + leaf[3:6].astype(np.float64) * size - eps
    hi = lo + size + 2 * eps
    te, tx = -np.inf, np.inf
    for a in range(3):
        if direction[a] == 0.0:
            if not (lo[a] <= origin[a] <= hi[a]):
                return np.inf, -np.inf
            continue
        t0 = (lo[a] - origin[a]) / direction[a]
        t1 = (hi[a] - origin[a]) / direction[a]
        te = max(te, min(t0, t1))
        tx = min(tx, max(t0, t1))
    return max(te, 0.0), tx
