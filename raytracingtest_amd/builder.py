"""SVO builder: surface leaves -> compact node pool in the reference layout.

Restates the compression half of NaiveCreator (Assets/Scripts/SVO/CompactSVO/
NaiveCreator.cs) level-parallel instead of by recursion:

  * tree build (BuildTree :52-118): a node exists iff some leaf below it is a
    surface voxel; internal normal = Normalize(sum of child normals, child
    order 0..7); internal colour = (mean of the children's colour.r, 0, 0)
    (the reference only sums color.r, :105);
  * layout (CompressSVO / CompressSVOAux :132-193): descriptors in the order
    the recursion appends them -- a node's non-leaf children are appended as
    one contiguous block when the node is visited, visits are pre-order.  Here
    the block start of node n is 1 + (sum of block sizes of the nodes before n
    in pre-order), computed with one prefix sum over the pre-order;
  * descriptor = ptr16 << 16 | valid8 << 8 | nonleaf8 (:184-187), ptr relative;
  * attachment (GetAttachment :195-257): 565 colours A/B, 2-bit choices per
    child, encodeRawNormal16 (:547-571) of the node normal.

Float arithmetic follows the C# code in float32 (Unity Vector3 semantics).
The result is V1 (int32 descriptors) when every relative pointer fits 16 bits,
else V2 (uint64 nodes with absolute first-child index).

Leaf generators: Menger sponge here; density samplers
(NaiveCreator + SampleFunctions.cs) in the native builder (libsvo_build.so).
"""
import numpy as np

from .svo_data import SVOData

F = np.float32


def _part1by2(v):
    v = v.astype(np.uint64) & np.uint64(0x1FFFFF)
    v = (v | (v << np.uint64(32))) & np.uint64(0x1F00000000FFFF)
    v = (v | (v << np.uint64(16))) & np.uint64(0x1F0000FF0000FF)
    v = (v | (v << np.uint64(8))) & np.uint64(0x100F00F00F00F00F)
    v = (v | (v << np.uint64(4))) & np.uint64(0x10C30C30C30C30C3)
    v = (v | (v << np.uint64(2))) & np.uint64(0x1249249249249249)
    return v


def morton(xyz):
    """Child slot c = x | y << 1 | z << 2 at every level (Constants.cs:23-26)."""
    xyz = np.asarray(xyz)
    return _part1by2(xyz[:, 0]) | (_part1by2(xyz[:, 1]) << np.uint64(1)) | (_part1by2(xyz[:, 2]) << np.uint64(2))


def normalize_unity(v):
    """Vector3.Normalize: mag = sqrt(x*x + y*y + z*z) (float), v / mag if mag > 1e-5 else 0."""
    v = np.asarray(v, F)
    sq = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
    mag = np.sqrt(sq.astype(F)).astype(F)
    ok = mag > F(1e-5)
    safe = np.where(ok, mag, F(1)).astype(F)
    out = (v / safe[:, None]).astype(F)
    return np.where(ok[:, None], out, F(0)).astype(F)


def _to_int_trunc(x):
    """C# (int) cast of a float: truncation; NaN / out of range -> int.MinValue."""
    x = np.asarray(x, np.float64)
    bad = ~np.isfinite(x) | (x >= 2147483648.0) | (x < -2147483648.0)
    return np.where(bad, -2147483648, np.trunc(np.where(bad, 0, x))).astype(np.int64)


def encode_raw_normal16(n):
    """NaiveCreator.encodeRawNormal16 (NaiveCreator.cs:547-571), vectorised, float32."""
    n = np.asarray(n, F)
    a = np.abs(n)
    axis = np.where(a[:, 0] >= np.maximum(a[:, 1], a[:, 2]), 0, np.where(a[:, 1] >= a[:, 2], 1, 2))
    t = np.where(axis == 0, n[:, 0], np.where(axis == 1, n[:, 1], n[:, 2]))
    u = np.where(axis == 0, n[:, 1], np.where(axis == 1, n[:, 2], n[:, 0]))
    v = np.where(axis == 0, n[:, 2], np.where(axis == 1, n[:, 0], n[:, 1]))
    sign = np.where(t >= F(0), 0, 0x8000)
    with np.errstate(divide="ignore", invalid="ignore"):
        at = np.abs(t).astype(F)
        fu = ((u / at).astype(F) * F(63.0)).astype(F)
        fv = ((v / at).astype(F) * F(31.0)).astype(F)
    # Mathf.Clamp keeps NaN (neither comparison holds)
    fu = np.where(fu < -64, F(-64), np.where(fu > 63, F(63), fu))
    fv = np.where(fv < -32, F(-32), np.where(fv > 31, F(31), fv))
    iu = (_to_int_trunc(fu) & 0x7F) << 6
    iv = _to_int_trunc(fv) & 0x3F
    return (sign | (axis << 13) | iu | iv).astype(np.uint32) & 0xFFFF


def compress_color(c):
    """NaiveCreator.CompressColor (NaiveCreator.cs:351-356)."""
    c = np.asarray(c, F)
    r = _to_int_trunc((F(32) * (c[:, 0] - F(0.00001))).astype(F))
    g = _to_int_trunc((F(64) * (c[:, 1] - F(0.00001))).astype(F))
    b = _to_int_trunc((F(32) * (c[:, 2] - F(0.00001))).astype(F))
    return (r | (g << 5) | (b << 11)) & 0xFFFFFFFF


def _distance(a, b):
    d = (a - b).astype(F)
    sq = ((d[..., 0] * d[..., 0]).astype(F) + (d[..., 1] * d[..., 1]).astype(F)).astype(F)
    sq = (sq + (d[..., 2] * d[..., 2]).astype(F)).astype(F)
    return np.sqrt(sq).astype(F)


def attachments_for(child_present, child_color, node_normal):
    """GetAttachment (NaiveCreator.cs:195-257) for many nodes at once.
    child_present: bool[N, 8]; child_color: float32[N, 8, 3]; node_normal: float32[N, 3].
    Returns uint32[N, 2] = (A | B << 16, choices | normal16 << 16)."""
    n = len(child_present)
    A = np.zeros((n, 3), F)
    B = np.zeros((n, 3), F)
    seen = np.zeros(n, bool)
    for i in range(8):
        p = child_present[:, i]
        first = p & ~seen
        A[first] = child_color[first, i]
        later = p & seen
        if later.any():
            # bdist never updates in the reference (stays 0): B = last child differing from A
            dist = _distance(A, child_color[:, i])
            upd = later & (dist > F(0))
            B[upd] = child_color[upd, i]
        seen |= p
    cand = np.stack([A, B, (F(0.667) * A + F(0.333) * B).astype(F), (F(0.333) * A + F(0.667) * B).astype(F)], axis=1)
    choices = np.zeros(n, np.int64)
    for i in range(8):
        p = child_present[:, i]
        if not p.any():
            continue
        best = np.full(n, F(100))
        choice = np.zeros(n, np.int64)
        for j in range(4):
            dist = _distance(child_color[:, i], cand[:, j])
            better = dist < best
            best = np.where(better, dist, best)
            choice = np.where(better, j, choice)
        choices |= np.where(p, choice << (2 * i), 0)
    ca = compress_color(A)
    cb = compress_color(B)
    nrm = encode_raw_normal16(node_normal)
    lo = (ca | (cb << 16)) & 0xFFFFFFFF
    hi = (choices | (nrm.astype(np.int64) << 16)) & 0xFFFFFFFF
    return np.stack([lo, hi], axis=1).astype(np.uint32)


def build_from_leaves(depth, leaf_xyz, leaf_normal, leaf_color=None):
    """Compact SVO from surface leaves at integer coordinates of a 2^depth grid.

    leaf_color defaults to the reference's node.color = position - 1
    (NaiveCreator.cs:66), i.e. xyz / 2^depth."""
    depth = int(depth)
    if not 1 <= depth <= 21:
        raise ValueError("depth must be in [1, 21]")
    xyz = np.asarray(leaf_xyz, np.int64)
    if len(xyz) == 0:
        return SVOData(childDescriptors=np.zeros(1, np.int32))
    code = morton(xyz)
    order = np.argsort(code, kind="stable")
    code = code[order]
    if np.any(code[1:] == code[:-1]):
        raise ValueError("duplicate leaf coordinates")
    nrm = np.asarray(leaf_normal, F)[order]
    if leaf_color is None:
        col = (xyz[order].astype(F) * F(1.0 / (1 << depth))).astype(F)
    else:
        col = np.asarray(leaf_color, F)[order]

    # bottom-up: level k has keys = code >> 3 (depth - k); level `depth` = leaves
    keys = [None] * (depth + 1)
    normals = [None] * (depth + 1)
    colors = [None] * (depth + 1)
    keys[depth], normals[depth], colors[depth] = code, nrm, col
    valid = [None] * depth
    present = [None] * depth
    ccolor = [None] * depth
    for k in range(depth - 1, -1, -1):
        ck = keys[k + 1]
        pk = ck >> np.uint64(3)
        uk, start = np.unique(pk, return_index=True)
        parent_of = np.searchsorted(uk, pk)
        slot = (ck & np.uint64(7)).astype(np.int64)
        m = len(uk)
        pres = np.zeros((m, 8), bool)
        pres[parent_of, slot] = True
        cc = np.zeros((m, 8, 3), F)
        cc[parent_of, slot] = colors[k + 1]
        cn = np.zeros((m, 8, 3), F)
        cn[parent_of, slot] = normals[k + 1]
        s = np.zeros((m, 3), F)
        for i in range(8):                       # normal += child.normal, in child order
            s = (s + cn[:, i]).astype(F)
        normals[k] = normalize_unity(s)
        r = np.zeros(m, F)
        for i in range(8):                       # color.x += child.color.r
            r = (r + cc[:, i, 0]).astype(F)
        cnt = pres.sum(axis=1).astype(F)
        inv = (F(1) / cnt).astype(F)
        colors[k] = np.stack([(r * inv).astype(F), np.zeros(m, F), np.zeros(m, F)], axis=1)
        keys[k] = uk
        valid[k] = (pres * (1 << np.arange(8))).sum(axis=1).astype(np.uint32)
        present[k] = pres
        ccolor[k] = cc

    # pre-order of internal nodes: sort by (key padded to level depth-1, level)
    counts = [len(keys[k]) for k in range(depth)]
    lvl = np.concatenate([np.full(c, k, np.int64) for k, c in enumerate(counts)])
    padded = np.concatenate([keys[k] << np.uint64(3 * (depth - 1 - k)) for k in range(depth)])
    local = np.concatenate([np.arange(c) for c in counts])
    pre = np.lexsort((lvl, padded))
    nonleaf = [valid[k] if k < depth - 1 else np.zeros(counts[k], np.uint32) for k in range(depth)]
    kcount = np.concatenate([np.array([bin(v).count("1") for v in range(256)], np.int64)[nonleaf[k]]
                             for k in range(depth)])
    block_pre = 1 + np.concatenate([[0], np.cumsum(kcount[pre])[:-1]])
    block = np.empty_like(block_pre)
    block[pre] = block_pre                     # block start per (level-major) node
    offs = np.concatenate([[0], np.cumsum(counts)])

    index = np.zeros(offs[-1], np.int64)
    for k in range(depth - 1):                 # children get block(parent) + rank among siblings
        ck = keys[k + 1]
        parent = np.searchsorted(keys[k], ck >> np.uint64(3))
        first_child = np.concatenate([[True], (ck[1:] >> np.uint64(3)) != (ck[:-1] >> np.uint64(3))])
        grp = np.cumsum(first_child) - 1
        starts = np.flatnonzero(first_child)
        rank = np.arange(len(ck)) - starts[grp]
        index[offs[k + 1]:offs[k + 2]] = block[offs[k] + parent] + rank

    n = offs[-1]
    lo_all = np.zeros(n, np.uint32)
    first_all = np.zeros(n, np.uint64)
    att = np.zeros((n, 2), np.uint32)
    for k in range(depth):
        sl = slice(offs[k], offs[k + 1])
        ix = index[sl]
        lo_all[ix] = (valid[k] << 8) | nonleaf[k]
        first_all[ix] = np.where(nonleaf[k] != 0, block[sl], 0).astype(np.uint64)
        att[ix] = attachments_for(present[k], ccolor[k], normals[k])
    nodes = (first_all << np.uint64(32)) | lo_all.astype(np.uint64)
    data = SVOData(nodes=nodes, attachments=att.reshape(-1))
    try:
        return data.to_v1()
    except Exception:
        return data


# --------------------------------------------------------------------- leaves
def menger_solid(n, levels=5):
    """Menger sponge occupancy of an n^3 grid: voxel centre c = (i + 0.5) / n is
    solid unless, for some l in 1..levels, at least two axes have base-3 digit
    floor(c * 3^l) mod 3 == 1."""
    c = (np.arange(n) + 0.5) / n
    holes = np.zeros((n, n, n), bool)
    for l in range(1, levels + 1):
        d = (np.floor(c * 3 ** l).astype(np.int64) % 3) == 1
        cnt = d[:, None, None].astype(np.int8) + d[None, :, None] + d[None, None, :]
        holes |= cnt >= 2
    return ~holes   # indexed [x, y, z]


def surface_leaves(solid):
    """Solid voxels with an empty 6-neighbour (IsEdge, NaiveCreator.cs:121-130);
    outside the grid counts as empty.  Normal = normalised sum of the outward
    directions of the empty neighbours."""
    s = np.pad(solid, 1, constant_values=False)
    core = s[1:-1, 1:-1, 1:-1]
    nrm = np.zeros(core.shape + (3,), F)
    edge = np.zeros(core.shape, bool)
    for axis in range(3):
        for sgn in (1, -1):
            sl = [slice(1, -1)] * 3
            sl[axis] = slice(1 + sgn, s.shape[axis] - 1 + sgn)
            empty = ~s[tuple(sl)]
            edge |= empty
            nrm[..., axis] += np.where(empty, F(sgn), F(0))
    surf = core & edge
    xyz = np.argwhere(surf)
    normal = normalize_unity(nrm[surf])
    return xyz, normal


def build_menger(depth=8, levels=5):
    n = 1 << depth
    xyz, normal = surface_leaves(menger_solid(n, levels))
    return build_from_leaves(depth, xyz, normal)


def build_svo_for_sampler(sample_type, max_level):
    """RaytracingMaster.SetSVOBuffer() path: NaiveCreator.Create(SampleFunctions.functions[t], maxLevel)."""
    from .native_builder import build_sampler_svo
    return build_sampler_svo(sample_type, max_level)


# ------------------------------------------------------------ leaf linking
def link_leaves(svo, get_leaf):
    """NaiveCreator.Create(root, getLeaf) (NaiveCreator.cs:30-42, :156-159) on a
    built pool: every leaf child becomes a link into a separately uploaded
    sub-SVO (Clipmap.UpdateMasterOctree, Clipmap.cs:153-169, links every chunk
    leaf to one sphere SVO uploaded at descriptor 10000).  The child keeps its
    valid bit and loses its leaf bit (the traversal descends into it); the
    node's child pointer is get_leaf(child) - node for the LAST leaf child in
    slot order (the reference overwrites it per leaf child), so linked child k
    of a node lands on descriptor target + rank(k).

    get_leaf(ix, iy, iz, level) -> absolute descriptor index (the reference
    passes the child's (int)position and size; see oracle/naive_creator.py).
    A node holding both leaf and non-leaf children cannot be linked (the
    reference would lay the non-leaf children out at the link target) and is
    rejected.  Returns a new SVOData (V1 when every pointer fits 16 bits)."""
    lo, first = svo.masks_and_first()
    valid = (lo >> 8) & 0xFF
    nonleaf = lo & 0xFF
    leaves = svo.leaf_voxels()                      # (node, slot, L, ix, iy, iz)
    if len(leaves) == 0:
        return svo
    nodes = np.unique(leaves[:, 0])
    mixed = nodes[nonleaf[nodes] != 0]
    if len(mixed):
        raise ValueError(f"node {int(mixed[0])} holds leaf and non-leaf children: cannot link its leaves")
    # last leaf child of every node (slot order)
    order = np.lexsort((leaves[:, 1], leaves[:, 0]))
    rows = leaves[order]
    last = np.concatenate([rows[1:, 0] != rows[:-1, 0], [True]])
    new_lo = lo.copy()
    new_first = first.astype(np.int64).copy()
    for r in rows[last]:
        node = int(r[0])
        target = int(get_leaf(int(r[3]), int(r[4]), int(r[5]), int(r[2]) + 1))
        if target <= node or target >= 1 << 32:
            raise ValueError(f"link target {target} of node {node} must lie after the node")
        new_lo[node] = (valid[node] << 8) | valid[node]
        new_first[node] = target
    nodes_v2 = (new_first.astype(np.uint64) << np.uint64(32)) | new_lo.astype(np.uint64)
    data = SVOData(nodes=nodes_v2, attachments=svo.attachments.copy())
    try:
        return data.to_v1()
    except Exception:
        return data
