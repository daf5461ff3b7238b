"""Loader for the native C-ABI library libsvo_rt.so (include/svo_rt.h).

The product path has no CPU fallback: if the HIP library is missing or cannot
be loaded, every entry point raises.  torch is imported first when available
so that the process holds ONE HIP runtime (torch's libamdhip64.so.7 and
/opt/rocm's share the soname; whichever loads first is used by both).
"""
import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# SVO_RT_LIB: diagnostics only -- another build of this same library (tools/ab_lib.sh
# compiles variants under build/ab/ and A/B-tests them in one GPU session)
LIB_PATH = os.environ.get("SVO_RT_LIB") or os.path.join(PKG_DIR, "libsvo_rt.so")
BUILDER_PATH = os.path.join(PKG_DIR, "libsvo_build.so")

SVO_OK = 0
STACK_HLSL, STACK_EXACT = 0, 1

HIT_DTYPE = np.dtype([("parent", "<u4"), ("hit_idx", "u1"), ("hit_scale", "u1"),
                      ("flags", "<u2"), ("t", "<f4"), ("nx", "<f4"), ("ny", "<f4"),
                      ("nz", "<f4")])
assert HIT_DTYPE.itemsize == 24

# every symbol include/svo_rt.h declares
EXPORTS = ("svo_create", "svo_set_buffer", "svo_set_buffer_v2", "svo_set_camera", "svo_render",
           "svo_render_device", "svo_count_fetches", "svo_get_info", "svo_synchronize",
           "svo_destroy", "svo_last_error", "svo_abi_version", "svo_set_options", "svo_accumulate",
           "svo_kernel_time")
SVO_OPT_SHADOW_RAYS = 1
SVO_OPT_KERNEL_TIMING = 2


class SvoBand(ctypes.Structure):
    _fields_ = [("band_rows", ctypes.c_int), ("band_rank", ctypes.c_int),
                ("band_count", ctypes.c_int)]


class SvoError(RuntimeError):
    pass


_lib = None


def _load_torch_first():
    try:
        import torch  # noqa: F401
    except Exception:  # torch is plumbing only; the C-ABI does not need it
        pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SvoError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    _load_torch_first()
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    vp, sz, i, f = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_float
    L.svo_create.argtypes = [i, sz, ctypes.POINTER(vp)]
    L.svo_set_buffer.argtypes = [vp, vp, sz, vp, sz, sz]
    L.svo_set_buffer_v2.argtypes = [vp, vp, sz, vp, sz, sz]
    L.svo_set_camera.argtypes = [vp, vp, vp, f, f, vp]
    L.svo_render.argtypes = [vp, i, i, i, vp, vp]
    L.svo_render_device.argtypes = [vp, i, i, i, vp, vp, vp, vp]
    L.svo_count_fetches.argtypes = [vp, i, i, i, vp, vp, vp]
    L.svo_set_options.argtypes = [vp, ctypes.c_uint32]
    L.svo_kernel_time.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
    L.svo_accumulate.argtypes = [vp, vp, vp, sz, ctypes.c_uint32, vp]
    L.svo_get_info.argtypes = [vp, ctypes.POINTER(sz), ctypes.POINTER(i), ctypes.POINTER(i)]
    L.svo_synchronize.argtypes = [vp]
    L.svo_destroy.argtypes = [vp]
    L.svo_last_error.restype = ctypes.c_char_p
    L.svo_last_error.argtypes = []
    L.svo_abi_version.restype = i
    for name in EXPORTS:
        getattr(L, name).restype = getattr(L, name).restype or i
    L.svo_last_error.restype = ctypes.c_char_p
    _lib = L
    return L


def check(rc, what):
    if rc != SVO_OK:
        msg = lib().svo_last_error().decode(errors="replace")
        raise SvoError(f"{what} failed ({rc}): {msg}")
