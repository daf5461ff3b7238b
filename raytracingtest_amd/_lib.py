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

COMPACT_DTYPE = np.dtype([("parent", "<u4"), ("meta", "<u4"), ("t", "<f4")])   # svo_hit_compact
assert COMPACT_DTYPE.itemsize == 12

ABI_VERSION = 10
# every symbol include/svo_rt.h declares
EXPORTS = ("svo_create", "svo_set_buffer", "svo_set_buffer_v2", "svo_set_camera", "svo_render",
           "svo_render_device", "svo_count_fetches", "svo_get_info", "svo_synchronize",
           "svo_destroy", "svo_last_error", "svo_abi_version", "svo_set_options", "svo_accumulate",
           "svo_kernel_time", "svo_create_multi", "svo_num_devices", "svo_get_member", "svo_render_frame",
           "svo_assemble_frame", "svo_stage_time", "svo_render_progressive", "svo_set_band_deal",
           "svo_pack_hits", "svo_get_member_link", "svo_stage_times", "svo_render_samples",
           "svo_render_progressive_async", "svo_progressive_last", "svo_forget_stream", "svo_get_config",
           "svo_set_config", "svo_beam_starts")
SVO_OPT_SHADOW_RAYS = 1
SVO_OPT_KERNEL_TIMING = 2
SVO_OPT_COUNT_BEAM = 4
LAYOUT_BAND, LAYOUT_FRAME = 0, 1
PART_COMPACT, PART_RGBA8, PART_RGB8, PART_SPARSE_RGB8 = 0, 1, 2, 3
LINK_SELF, LINK_PEER, LINK_COPY = 0, 1, 2
LINK_NAMES = {LINK_SELF: "self", LINK_PEER: "xgmi_peer_pull", LINK_COPY: "peer_copy"}


def sparse_head_bytes(n_tiles):
    """SVO_SPARSE_HEAD_BYTES: tile masks + tile offsets + count of a sparse part;
    the band's hit count is the uint32 at byte 12 * n_tiles."""
    return 12 * n_tiles + 4


def sparse_part_bytes(n_tiles, n_px):
    """SVO_SPARSE_PART_BYTES: capacity of a sparse part (every pixel a hit, plus
    the scan's scratch tail)."""
    return ((sparse_head_bytes(n_tiles) + 3 * n_px + 3) & ~3) + 4 * n_tiles + 4 * ((n_tiles + 1023) // 1024)
STAGE_KERNEL, STAGE_ASSEMBLE = 0, 1
MAX_SAMPLES = 8   # svo_render_samples: jittered samples per launch
PIXELS_RGBA8, PIXELS_RGB8 = 0, 1   # svo_render_progressive_async pixel formats


class SvoBand(ctypes.Structure):
    _fields_ = [("band_rows", ctypes.c_int), ("band_rank", ctypes.c_int),
                ("band_count", ctypes.c_int), ("cycle", ctypes.c_int),
                ("owner", ctypes.POINTER(ctypes.c_uint8))]


def make_band(band):
    """svo_band of a Python deal: (band_rows, band_rank, band_count) round-robin, or
    (band_rows, band_rank, band_count, owner) with owner[b % len(owner)] = rank
    of band b.  The struct keeps its owner array alive."""
    if len(band) == 3:
        return SvoBand(int(band[0]), int(band[1]), int(band[2]), 0, None)
    owner = (ctypes.c_uint8 * len(band[3]))(*[int(o) for o in band[3]])
    b = SvoBand(int(band[0]), int(band[1]), int(band[2]), len(band[3]),
                ctypes.cast(owner, ctypes.POINTER(ctypes.c_uint8)))
    b._owner = owner
    return b


class SvoFrame(ctypes.Structure):
    """svo_frame: device pointers (ints) of every per-pixel output, each nullable."""
    _fields_ = [("hits", ctypes.c_void_p), ("rgba", ctypes.c_void_p), ("rgba8", ctypes.c_void_p),
                ("compact", ctypes.c_void_p), ("position", ctypes.c_void_p), ("voxel", ctypes.c_void_p),
                ("rgb8", ctypes.c_void_p), ("hitmask", ctypes.c_void_p), ("layout", ctypes.c_int)]


# svo_config (include/svo_rt.h, ABI 10): the context's render policy, versioned by size
CONFIG_VERSION = 2   # 2: beam_back_held appended
_i32, _u32, _f32 = ctypes.c_int32, ctypes.c_uint32, ctypes.c_float
CONFIG_FIELDS = [
    ("tile_order", _i32), ("xcd_strips", _i32), ("issue_priority", _i32), ("order_every", _i32),
    ("move_every", _i32), ("move_spread", _i32), ("relayout", _i32), ("fetch_all", _i32),
    ("loop_form", _i32), ("lat_ratio", _f32),
    ("segments", _i32), ("seg_table_latency", _u32), ("seg_table_issue", _u32), ("seg_table_thin", _u32),
    ("seg_ratio", _f32), ("seg_thin_ratio", _f32), ("seg_cap", _i32), ("seg_min_chain", _i32),
    ("seg_move", _i32), ("seg_jitter", _i32), ("seg_all", _i32), ("seg_scramble", _u32),
    ("beam", _i32), ("beam_back", _i32),
    ("shadow_form", _i32), ("shadow_order", _i32),
    ("readback", _i32), ("host_copy_threads", _i32),
    ("sparse_payload", _i32), ("peer_copy", _i32),
    ("beam_back_held", _i32)]   # version 2
SHADOW_FUSED, SHADOW_TILES, SHADOW_LIST = 0, 1, 2   # svo_config.shadow_form


class SvoConfig(ctypes.Structure):
    _fields_ = [("size", _u32), ("version", _u32)] + CONFIG_FIELDS

    def to_dict(self):
        return {name: getattr(self, name) for name, _ in CONFIG_FIELDS}


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
    sig = {
        "svo_create": [i, sz, ctypes.POINTER(vp)],
        "svo_set_buffer": [vp, vp, sz, vp, sz, sz],
        "svo_set_buffer_v2": [vp, vp, sz, vp, sz, sz],
        "svo_set_camera": [vp, vp, vp, f, f, vp],
        "svo_render": [vp, i, i, i, vp, vp],
        "svo_render_device": [vp, i, i, i, vp, vp, vp, vp],
        "svo_count_fetches": [vp, i, i, i, vp, vp, vp],
        "svo_set_options": [vp, ctypes.c_uint32],
        "svo_kernel_time": [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)],
        "svo_accumulate": [vp, vp, vp, sz, ctypes.c_uint32, vp],
        "svo_get_info": [vp, ctypes.POINTER(sz), ctypes.POINTER(i), ctypes.POINTER(i)],
        "svo_create_multi": [ctypes.POINTER(i), i, sz, i, ctypes.POINTER(vp)],
        "svo_num_devices": [vp, ctypes.POINTER(i)],
        "svo_get_member": [vp, i, ctypes.POINTER(vp)],
        "svo_get_member_link": [vp, i, ctypes.POINTER(i), ctypes.POINTER(i)],
        "svo_render_frame": [vp, i, i, i, vp, ctypes.POINTER(SvoFrame), vp],
        "svo_assemble_frame": [vp, i, i, ctypes.POINTER(SvoBand), i, ctypes.POINTER(vp), i, i,
                               ctypes.POINTER(SvoFrame), vp],
        "svo_stage_time": [vp, i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)],
        "svo_stage_times": [vp, i, ctypes.POINTER(f), sz, ctypes.POINTER(sz)],
        "svo_render_samples": [vp, i, i, i, ctypes.POINTER(SvoBand), i, ctypes.POINTER(f), ctypes.c_uint32, vp, vp, vp,
                               i, vp],
        "svo_render_progressive": [vp, i, i, i, ctypes.c_uint32, vp, vp],
        "svo_render_progressive_async": [vp, i, i, i, ctypes.c_uint32, i, ctypes.POINTER(vp)],
        "svo_progressive_last": [vp, ctypes.POINTER(vp)],
        "svo_set_band_deal": [vp, i, ctypes.POINTER(ctypes.c_uint8)],
        "svo_pack_hits": [vp, i, i, ctypes.POINTER(SvoBand), vp, vp, vp],
        "svo_synchronize": [vp],
        "svo_forget_stream": [vp, vp],
        "svo_get_config": [vp, ctypes.POINTER(SvoConfig)],
        "svo_set_config": [vp, ctypes.POINTER(SvoConfig)],
        "svo_beam_starts": [vp, i, i, ctypes.POINTER(SvoBand), vp, vp],
        "svo_destroy": [vp],
        "svo_last_error": [],
        "svo_abi_version": [],
    }
    # SVO_RT_LIB (A/B diagnostics) may name an older build: bind what it has
    strict = not os.environ.get("SVO_RT_LIB")
    for name in EXPORTS:
        if not strict and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.argtypes = sig[name]
        fn.restype = ctypes.c_char_p if name == "svo_last_error" else i
    _lib = L
    return L


def default_config():
    """svo_get_config(NULL): the library's defaults, as a dict of svo_config fields."""
    c = SvoConfig()
    c.size = ctypes.sizeof(SvoConfig)
    check(lib().svo_get_config(None, ctypes.byref(c)), "svo_get_config")
    return c.to_dict()


def check(rc, what):
    if rc != SVO_OK:
        msg = lib().svo_last_error().decode(errors="replace")
        raise SvoError(f"{what} failed ({rc}): {msg}")
