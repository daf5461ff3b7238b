"""ctypes front-end of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It loads oracle/build/liborcsvo.so (built by oracle/Makefile via
__graft_entry__.build()); see svo_oracle.h for what the C code restates and
how it is pinned.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liborcsvo.so")

FMT_V1, FMT_V2 = 1, 2
STACK_HLSL, STACK_EXACT = 0, 1
SHADOW_RAYS = 0x100   # OR into stack_mode: one shadow ray per primary hit
COUNT_ITERS = 0x200   # OR into stack_mode: the fetch output counts loop iterations instead
COUNT_SHADOW_ITERS = 0x400   # with SHADOW_RAYS: the fetch output counts the shadow ray's iterations

HIT_DTYPE = np.dtype([("parent", "<u4"), ("hit_idx", "u1"), ("hit_scale", "u1"),
                      ("flags", "<u2"), ("t", "<f4"), ("nx", "<f4"), ("ny", "<f4"),
                      ("nz", "<f4")])
assert HIT_DTYPE.itemsize == 24


class _Svo(ctypes.Structure):
    _fields_ = [("format", ctypes.c_int), ("desc", ctypes.c_void_p), ("nodes", ctypes.c_void_p),
                ("n_nodes", ctypes.c_size_t), ("att", ctypes.c_void_p)]


class _Cam(ctypes.Structure):
    _fields_ = [("c2w", ctypes.c_float * 16), ("inv_proj", ctypes.c_float * 16),
                ("px_off", ctypes.c_float * 2), ("light", ctypes.c_float * 4)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i, f = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_float
        L.orc_decode_normal.argtypes = [ctypes.c_uint32, vp]
        L.orc_decode_dxt_color.argtypes = [ctypes.c_uint32, ctypes.c_uint32, i, vp]
        L.orc_camera_ray.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, i, i, vp, vp]
        L.orc_intersect.argtypes = [vp, vp, vp, i, vp, vp, vp, vp]
        L.orc_intersect.restype = i
        L.orc_render.argtypes = [vp, vp, i, i, i, i, i, i, vp, vp, vp]
        L.orc_render_pixels.argtypes = [vp, vp, i, i, vp, sz, i, i, vp, vp, vp]
        L.orc_render_ex.argtypes = [vp, vp, i, i, i, i, i, i, vp, vp, vp, vp, vp]
        L.orc_pack_rgba8.argtypes = [vp, sz, vp]
        L.orc_v1_to_v2.argtypes = [vp, sz, vp]
        L.orc_accumulate.argtypes = [vp, vp, sz, ctypes.c_uint32]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


class OracleSVO:
    """Holds the arrays alive and the C descriptor struct."""

    def __init__(self, descriptors=None, attachments=None, nodes=None):
        if nodes is not None:
            self.nodes = np.ascontiguousarray(nodes, dtype=np.uint64)
            self.desc = None
            n = len(self.nodes)
            fmt = FMT_V2
        else:
            self.desc = np.ascontiguousarray(descriptors, dtype=np.int32)
            self.nodes = None
            n = len(self.desc)
            fmt = FMT_V1
        self.att = np.ascontiguousarray(attachments, dtype=np.uint32)
        assert len(self.att) >= 2 * n
        self.s = _Svo(fmt, _ptr(self.desc), _ptr(self.nodes), n, _ptr(self.att))


def make_camera(c2w, inv_proj, px_off=(0.5, 0.5), light=(0.0, -1.0, 0.0, 1.0)):
    """c2w / inv_proj: 4x4 float32 numpy arrays in mathematical (row, col) order."""
    cam = _Cam()
    cam.c2w[:] = np.asarray(c2w, np.float32).T.reshape(-1).tolist()       # column-major
    cam.inv_proj[:] = np.asarray(inv_proj, np.float32).T.reshape(-1).tolist()
    cam.px_off[:] = [float(np.float32(v)) for v in px_off]
    cam.light[:] = [float(np.float32(v)) for v in light]
    return cam


def decode_normal(code):
    out = np.zeros(3, np.float32)
    lib().orc_decode_normal(int(code), out.ctypes.data)
    return out


def decode_dxt_color(head, bits, texel):
    out = np.zeros(3, np.float32)
    lib().orc_decode_dxt_color(int(head), int(bits), int(texel), out.ctypes.data)
    return out


def camera_ray(cam, x, y, width, height):
    o = np.zeros(3, np.float32)
    d = np.zeros(3, np.float32)
    lib().orc_camera_ray(ctypes.byref(cam), x, y, width, height, o.ctypes.data, d.ctypes.data)
    return o, d


def intersect(svo, origin, direction, stack_mode=STACK_HLSL):
    o = np.ascontiguousarray(origin, np.float32)
    d = np.ascontiguousarray(direction, np.float32)
    hit = np.zeros(1, HIT_DTYPE)
    alb = np.zeros(3, np.float32)
    f = np.zeros(1, np.uint32)
    it = np.zeros(1, np.uint32)
    lib().orc_intersect(ctypes.byref(svo.s), o.ctypes.data, d.ctypes.data, stack_mode,
                        hit.ctypes.data, alb.ctypes.data, f.ctypes.data, it.ctypes.data)
    return hit[0], alb, int(f[0]), int(it[0])


def render(svo, cam, width, height, stack_mode=STACK_HLSL, y0=0, y1=None, nthreads=None,
           want_rgba=True, want_fetches=True):
    y1 = height if y1 is None else y1
    n = (y1 - y0) * width
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    hits = np.zeros(n, HIT_DTYPE)
    rgba = np.zeros((n, 4), np.float32) if want_rgba else None
    fet = np.zeros(n, np.uint32) if want_fetches else None
    lib().orc_render(ctypes.byref(svo.s), ctypes.byref(cam), width, height, y0, y1, stack_mode,
                     nthreads, hits.ctypes.data, _ptr(rgba), _ptr(fet))
    return hits, rgba, fet


def render_ex(svo, cam, width, height, stack_mode=STACK_HLSL, y0=0, y1=None, nthreads=None):
    """render() plus per-pixel bestHit.position (float4, w = 0) and voxel keys."""
    y1 = height if y1 is None else y1
    n = (y1 - y0) * width
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    hits = np.zeros(n, HIT_DTYPE)
    rgba = np.zeros((n, 4), np.float32)
    fet = np.zeros(n, np.uint32)
    pos = np.zeros((n, 4), np.float32)
    vox = np.zeros(n, np.uint64)
    lib().orc_render_ex(ctypes.byref(svo.s), ctypes.byref(cam), width, height, y0, y1, stack_mode, nthreads,
                        hits.ctypes.data, rgba.ctypes.data, fet.ctypes.data, pos.ctypes.data, vox.ctypes.data)
    return hits, rgba, fet, pos, vox


def pack_rgba8(rgba):
    """Display RGBA8 words of RGBA32F pixels (svo_frame.rgba8)."""
    rgba = np.ascontiguousarray(rgba, np.float32).reshape(-1, 4)
    out = np.zeros(len(rgba), np.uint32)
    lib().orc_pack_rgba8(rgba.ctypes.data, len(rgba), out.ctypes.data)
    return out


def render_pixels(svo, cam, width, height, pixels, stack_mode=STACK_HLSL, nthreads=None,
                  want_rgba=True):
    pixels = np.ascontiguousarray(pixels, np.uint32)
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    n = len(pixels)
    hits = np.zeros(n, HIT_DTYPE)
    rgba = np.zeros((n, 4), np.float32) if want_rgba else None
    fet = np.zeros(n, np.uint32)
    lib().orc_render_pixels(ctypes.byref(svo.s), ctypes.byref(cam), width, height,
                            pixels.ctypes.data, n, stack_mode, nthreads, hits.ctypes.data,
                            _ptr(rgba), fet.ctypes.data)
    return hits, rgba, fet


def v1_to_v2(desc):
    desc = np.ascontiguousarray(desc, np.int32)
    out = np.zeros(len(desc), np.uint64)
    lib().orc_v1_to_v2(desc.ctypes.data, len(desc), out.ctypes.data)
    return out


def accumulate(dst, src, sample):
    """In-place AddShader blend of float32 RGBA frames (any shape [..., 4])."""
    assert dst.dtype == np.float32 and src.dtype == np.float32 and dst.shape == src.shape
    assert dst.flags.c_contiguous and src.flags.c_contiguous
    lib().orc_accumulate(dst.ctypes.data, src.ctypes.data, dst.size // 4, int(sample))
    return dst
