"""ctypes front-end of libsvo_build.so (include/svo_build.h): the native
restatement of NaiveCreator (Assets/Scripts/SVO/CompactSVO/NaiveCreator.cs)
with GPU leaf classification."""
import ctypes
import os

import numpy as np

from ._lib import BUILDER_PATH, SvoError, _load_torch_first
from .svo_data import SVOData

# SampleFunctions.Type (SampleFunctions.cs:4-11)
FLAT_GROUND, SPHERE, SIMPLEX, ROTATED_CUBOID, CUSTOM1 = range(5)


class _Result(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_size_t), ("depth", ctypes.c_int), ("v1_ok", ctypes.c_int),
                ("descriptors", ctypes.POINTER(ctypes.c_int32)), ("nodes", ctypes.POINTER(ctypes.c_uint64)),
                ("attachments", ctypes.POINTER(ctypes.c_uint32)), ("n_leaves", ctypes.c_size_t)]


_blib = None


def blib():
    global _blib
    if _blib is None:
        if not os.path.exists(BUILDER_PATH):
            raise SvoError(f"{BUILDER_PATH} is not built: run __graft_entry__.build()")
        _load_torch_first()
        L = ctypes.CDLL(BUILDER_PATH, mode=ctypes.RTLD_GLOBAL)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.svob_build_sampler.argtypes = [i, i, i, ctypes.POINTER(_Result)]
        L.svob_build_from_leaves.argtypes = [i, sz, vp, vp, vp, ctypes.POINTER(_Result)]
        L.svob_surface_leaves.argtypes = [i, i, i, ctypes.POINTER(sz), ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.svob_eval_sampler.argtypes = [i, sz, vp, vp]
        L.svob_opensimplex_table.argtypes = [vp]
        L.svob_free.argtypes = [ctypes.POINTER(_Result)]
        L.svob_free.restype = None
        L.svob_free_ptr.argtypes = [vp]
        L.svob_free_ptr.restype = None
        L.svob_last_error.restype = ctypes.c_char_p
        for name in ("svob_build_sampler", "svob_build_from_leaves", "svob_surface_leaves", "svob_eval_sampler",
                     "svob_opensimplex_table"):
            getattr(L, name).restype = i
        _blib = L
    return _blib


def _check(rc, what):
    if rc != 0:
        raise SvoError(f"{what} failed ({rc}): {blib().svob_last_error().decode(errors='replace')}")


def _to_svodata(res, prefer_v1=True):
    n = res.n_nodes
    att = np.ctypeslib.as_array(res.attachments, shape=(2 * n,)).copy()
    if prefer_v1 and res.v1_ok:
        desc = np.ctypeslib.as_array(res.descriptors, shape=(n,)).copy()
        return SVOData(childDescriptors=desc, attachments=att)
    nodes = np.ctypeslib.as_array(res.nodes, shape=(n,)).copy()
    return SVOData(nodes=nodes, attachments=att)


def build_sampler_svo(sample_type, max_level, device=0, prefer_v1=True):
    """NaiveCreator.Create(SampleFunctions.functions[sample_type], max_level)."""
    res = _Result()
    _check(blib().svob_build_sampler(int(device), int(sample_type), int(max_level), ctypes.byref(res)),
           "svob_build_sampler")
    try:
        data = _to_svodata(res, prefer_v1)
        data.n_leaves = int(res.n_leaves)
        return data
    finally:
        blib().svob_free(ctypes.byref(res))


def build_from_leaves(depth, xyz, normals, colors=None, prefer_v1=True):
    """CompressSVO over given surface leaves (native twin of builder.build_from_leaves)."""
    xyz = np.ascontiguousarray(xyz, np.uint32).reshape(-1, 3)
    normals = np.ascontiguousarray(normals, np.float32).reshape(-1, 3)
    col = None if colors is None else np.ascontiguousarray(colors, np.float32).reshape(-1, 3)
    res = _Result()
    _check(blib().svob_build_from_leaves(int(depth), len(xyz), xyz.ctypes.data, normals.ctypes.data,
                                         None if col is None else col.ctypes.data, ctypes.byref(res)),
           "svob_build_from_leaves")
    try:
        return _to_svodata(res, prefer_v1)
    finally:
        blib().svob_free(ctypes.byref(res))


def surface_leaves(sample_type, max_level, device=0):
    """(Morton codes uint64[n], normals float32[n, 3]) of the surface voxels."""
    n = ctypes.c_size_t()
    mp = ctypes.c_void_p()
    npp = ctypes.c_void_p()
    _check(blib().svob_surface_leaves(int(device), int(sample_type), int(max_level), ctypes.byref(n),
                                      ctypes.byref(mp), ctypes.byref(npp)), "svob_surface_leaves")
    try:
        codes = np.ctypeslib.as_array(ctypes.cast(mp, ctypes.POINTER(ctypes.c_uint64)), shape=(n.value,)).copy() \
            if n.value else np.zeros(0, np.uint64)
        nrm = np.ctypeslib.as_array(ctypes.cast(npp, ctypes.POINTER(ctypes.c_float)), shape=(n.value, 3)).copy() \
            if n.value else np.zeros((0, 3), np.float32)
        return codes, nrm
    finally:
        blib().svob_free_ptr(mp)
        blib().svob_free_ptr(npp)


def eval_sampler(sample_type, xyz):
    xyz = np.ascontiguousarray(xyz, np.float32).reshape(-1, 3)
    out = np.zeros(len(xyz), np.float32)
    _check(blib().svob_eval_sampler(int(sample_type), len(xyz), xyz.ctypes.data, out.ctypes.data),
           "svob_eval_sampler")
    return out


def opensimplex_table():
    out = np.zeros((2048, 25), np.int8)
    _check(blib().svob_opensimplex_table(out.ctypes.data), "svob_opensimplex_table")
    return out


def table_digest(table):
    """sha256 of the canonical {hash: [count, offsets...]} listing."""
    import hashlib
    rows = []
    for h in range(2048):
        c = int(table[h, 0])
        if c:
            rows.append(f"{h}:" + ",".join(str(int(v)) for v in table[h, 1:1 + 3 * c]))
    return hashlib.sha256("\n".join(rows).encode()).hexdigest(), len(rows)
