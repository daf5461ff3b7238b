"""C-ABI boundary checks that need no GPU: the library builds, loads and exports
every symbol include/svo_rt.h declares; the header's record layout matches."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "svo_rt.h")


@pytest.fixture(scope="module")
def native():
    from raytracingtest_amd import build
    build.build()
    from raytracingtest_amd import _lib
    return _lib.lib()


def declared_functions(path):
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(svo_[a-z0-9_]+)\s*\(", text)))


def test_exports_every_declared_symbol(native):
    names = declared_functions(HEADER)
    assert len(names) >= 12
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "raytracingtest_amd", "libsvo_rt.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (svo_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    from raytracingtest_amd._lib import EXPORTS
    assert set(EXPORTS) == set(names)


def test_abi_version_and_error_text(native):
    from raytracingtest_amd import _lib
    assert native.svo_abi_version() == _lib.ABI_VERSION == 10
    assert isinstance(native.svo_last_error(), bytes)


def test_null_arguments_rejected_without_gpu(native):
    assert native.svo_create(0, 16, None) == -1        # SVO_ERR_ARG, no device touched
    assert b"null" in native.svo_last_error()
    assert native.svo_render(None, 8, 8, 0, None, None) == -1
    assert native.svo_destroy(None) == 0


def test_header_layout_compiles_in_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "svo_rt.h"\n#include <stddef.h>\n'
                   '_Static_assert(sizeof(svo_hit) == 24, "hit");\n'
                   '_Static_assert(offsetof(svo_hit, t) == 8, "t");\n'
                   '_Static_assert(offsetof(svo_hit, nz) == 20, "nz");\n'
                   '_Static_assert(sizeof(svo_band) == 16 + sizeof(void *), "band");\n'
                   '_Static_assert(sizeof(svo_hit_compact) == 12, "compact");\n'
                   '_Static_assert(offsetof(svo_frame, layout) == 64, "frame");\n'
                   '_Static_assert(SVO_PART_RGBA8 == 1 && SVO_PART_RGB8 == 2 && SVO_LAYOUT_FRAME == 1 && SVO_STAGE_ASSEMBLE == 1, "enums");\n'
                   'int main(void){return 0;}\n')
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src),
                    "-o", str(tmp_path / "t")], check=True)


def test_multi_device_and_frame_entry_points_reject_bad_arguments_without_gpu(native):
    import ctypes
    from raytracingtest_amd._lib import SvoFrame
    out = ctypes.c_void_p()
    assert native.svo_create_multi(None, 2, 16, 8, ctypes.byref(out)) == -1
    devs = (ctypes.c_int * 2)(0, 0)
    assert native.svo_create_multi(devs, 0, 16, 8, ctypes.byref(out)) == -1      # no device touched
    assert native.svo_create_multi(devs, 2, 16, 0, ctypes.byref(out)) == -1      # band_rows
    assert native.svo_render_frame(None, 8, 8, 0, None, ctypes.byref(SvoFrame()), None) == -1
    assert native.svo_assemble_frame(None, 8, 8, None, 1, None, 0, -1, None, None) == -1
    assert native.svo_stage_time(None, 0, None, None) == -1
    assert native.svo_set_band_deal(None, 0, None) == -1
    assert native.svo_pack_hits(None, 8, 8, None, None, None, None) == -1
    n = ctypes.c_int()
    assert native.svo_num_devices(None, ctypes.byref(n)) == -1


def test_compact_record_is_the_hit_record_prefix():
    from raytracingtest_amd import HIT_DTYPE
    from raytracingtest_amd._lib import COMPACT_DTYPE
    h = np.zeros(3, HIT_DTYPE)
    h["parent"] = [1, 0xFFFFFFFF, 7]
    h["hit_idx"], h["hit_scale"], h["flags"] = [5, 0, 2], [13, 0, 10], [9, 0, 1]
    h["t"] = [1.5, np.inf, 3.0]
    c = np.frombuffer(h.view(np.uint8).reshape(3, 24)[:, :12].tobytes(), COMPACT_DTYPE)
    assert np.array_equal(c["parent"], h["parent"]) and np.array_equal(c["t"], h["t"])
    assert np.array_equal(c["meta"], h["hit_idx"] | (h["hit_scale"].astype(np.uint32) << 8) |
                          (h["flags"].astype(np.uint32) << 16))


def test_sparse_part_sizes_match_header(tmp_path):
    """_lib.sparse_head_bytes / sparse_part_bytes == the header's SVO_SPARSE_* macros."""
    import subprocess
    src = tmp_path / "sizes.c"
    src.write_text('#include <stdio.h>\n#include "svo_rt.h"\nint main(void) {\n'
                   '  const int n[4][2] = {{0, 0}, {1, 7}, {1037, 66000}, {129600, 8294400}};\n'
                   '  for (int i = 0; i < 4; ++i) printf("%zu %zu\\n", (size_t)SVO_SPARSE_HEAD_BYTES(n[i][0]),\n'
                   '                                     (size_t)SVO_SPARSE_PART_BYTES(n[i][0], n[i][1]));\n'
                   '  return 0;\n}\n')
    exe = tmp_path / "sizes"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    from raytracingtest_amd import _lib
    for i, (nt, px) in enumerate([(0, 0), (1, 7), (1037, 66000), (129600, 8294400)]):
        assert int(out[2 * i]) == _lib.sparse_head_bytes(nt)
        assert int(out[2 * i + 1]) == _lib.sparse_part_bytes(nt, px)


def test_hit_dtype_matches_header():
    from raytracingtest_amd import HIT_DTYPE
    assert HIT_DTYPE.itemsize == 24
    assert HIT_DTYPE.fields["t"][1] == 8 and HIT_DTYPE.fields["nz"][1] == 20


def test_product_has_no_oracle_dependency():
    """The shipped package must never import or link the oracle."""
    pkg = os.path.join(ROOT, "raytracingtest_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(dirpath, f)).read()
                for pat in (r"^\s*(from|import)\s+oracle", r"liborcsvo", r"\borc_\w+\(", r"svo_oracle\.h"):
                    assert not re.search(pat, text, flags=re.M), (f, pat)


def test_unknown_option_bits_rejected_without_gpu(native):
    assert native.svo_set_options(None, 1) == -1          # null context
    from raytracingtest_amd._lib import SVO_OPT_KERNEL_TIMING, SVO_OPT_SHADOW_RAYS
    assert (SVO_OPT_SHADOW_RAYS, SVO_OPT_KERNEL_TIMING) == (1, 2)
    text = open(HEADER).read()
    assert "SVO_OPT_SHADOW_RAYS = 1" in text and "SVO_OPT_KERNEL_TIMING = 2" in text


def test_profile_key_does_not_depend_on_the_tree_location(tmp_path):
    """bench.py reads roofline.traffic from profiles/pmc_summary.json only when its
    source digest matches the running tree; the GPU box runs a scratch copy at
    another path, so the digest must not hash absolute paths."""
    import shutil
    import subprocess
    import sys
    dst = tmp_path / "copy"
    for d in ("raytracingtest_amd", "include"):
        shutil.copytree(os.path.join(ROOT, d), dst / d, ignore=shutil.ignore_patterns("*.so", "__pycache__"))
    code = "import sys; sys.path.insert(0, sys.argv[1]); from raytracingtest_amd.build import source_digest; print(source_digest())"
    here = subprocess.run([sys.executable, "-c", code, ROOT], capture_output=True, text=True, check=True).stdout
    there = subprocess.run([sys.executable, "-c", code, str(dst)], capture_output=True, text=True, check=True).stdout
    assert here.strip() and here == there


CONFIG_DEFAULTS = {
    "tile_order": 1, "xcd_strips": 1, "issue_priority": 1, "order_every": 32, "move_every": 4, "move_spread": 1,
    "relayout": 1, "fetch_all": -1, "loop_form": -1, "lat_ratio": 0.3, "segments": 1, "seg_table_latency": 0x444,
    "seg_table_issue": 0x4, "seg_table_thin": 0x888, "seg_ratio": 0.28, "seg_thin_ratio": 0.083, "seg_cap": 96,
    "seg_min_chain": 160, "seg_move": 2, "seg_jitter": 2, "seg_all": 0, "seg_scramble": 0, "beam": 1, "beam_back": 2,
    "shadow_form": 0, "shadow_order": 1, "readback": 0, "host_copy_threads": 0, "sparse_payload": 0, "peer_copy": 0,
    "beam_back_held": 0}


def test_config_struct_size_version_and_layout(tmp_path):
    """svo_config (ABI 10, config version 2): the ctypes mirror has the header's size, version and every field at the
    header's offset (the C# shim's StructLayout(Sequential) follows the same order)."""
    from raytracingtest_amd import _lib
    fields = [n for n, _ in _lib.CONFIG_FIELDS]
    src = tmp_path / "cfg.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "svo_rt.h"\nint main(void) {\n'
                   '  printf("%zu %d\\n", sizeof(svo_config), SVO_CONFIG_VERSION);\n' +
                   "".join(f'  printf("%zu\\n", offsetof(svo_config, {f}));\n' for f in fields) +
                   '  return 0;\n}\n')
    exe = tmp_path / "cfg"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                    str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(_lib.SvoConfig) == 132
    assert int(out[1]) == _lib.CONFIG_VERSION == 2
    for f, off in zip(fields, out[2:]):
        assert int(off) == getattr(_lib.SvoConfig, f).offset, f
    # every field is documented in INTEGRATION.md's config table and declared in the header
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    header = open(HEADER).read()
    for f in fields:
        assert f"`{f}`" in doc, f"INTEGRATION.md does not document {f}"
        assert re.search(rf"\b{f};", header), f


def test_config_defaults_and_size_versioning_without_gpu(native):
    """svo_get_config(NULL) gives the documented defaults (no device touched); a config smaller than
    size + version, or larger than this library's, is rejected; a shorter (older) struct is filled
    only up to its size."""
    from raytracingtest_amd import _lib
    got = _lib.default_config()
    for k, v in CONFIG_DEFAULTS.items():
        assert got[k] == pytest.approx(v), k
    assert set(got) == set(CONFIG_DEFAULTS)
    c = _lib.SvoConfig()
    c.size = 4
    assert native.svo_get_config(None, ctypes.byref(c)) == -1
    assert native.svo_set_config(None, ctypes.byref(c)) == -1
    # an older caller's struct: only the first 16 bytes (size, version, tile_order, xcd_strips)
    buf = (ctypes.c_uint8 * 132)(*([0xEE] * 132))
    hdr = ctypes.cast(buf, ctypes.POINTER(_lib.SvoConfig))
    hdr.contents.size = 16
    assert native.svo_get_config(None, hdr) == 0
    assert hdr.contents.size == 16 and hdr.contents.version == 2
    assert hdr.contents.tile_order == 1 and hdr.contents.xcd_strips == 1
    assert all(b == 0xEE for b in bytes(buf)[16:]), "wrote past the caller's size"
    # a version-1 caller (128 bytes, before beam_back_held): filled up to its size, the rest untouched
    hdr.contents.size = 128
    assert native.svo_get_config(None, hdr) == 0
    assert hdr.contents.size == 128 and hdr.contents.peer_copy == 0
    assert all(b == 0xEE for b in bytes(buf)[128:])


def test_library_reads_no_policy_from_the_environment():
    """policy travels in svo_config; the library's getenv calls are the four
    diagnostic switches (traces, the wave log, the splat's and the occupancy sweep's timing aids)."""
    names = []
    for f in ("svo_rt.hip", "svo_kernel.hip", "svo_build.hip"):
        text = open(os.path.join(ROOT, "raytracingtest_amd", "csrc", f)).read()
        names += re.findall(r"getenv\(\s*\"(\w+)\"", text)
        assert text.count("getenv(") == len(re.findall(r"getenv\(\s*\"\w+\"", text)), f
    assert sorted(names) == ["SVO_BEAM_DIAG", "SVO_DEBUG", "SVO_LDS_PAD", "SVO_WAVE_LOG"]


def test_csharp_shim_config_struct_follows_the_header():
    """unity/RaytracingMasterNative.cs's SvoConfig (StructLayout Sequential, no C# toolchain here to
    compile it) declares the header's fields in the header's order with 4-byte types."""
    from raytracingtest_amd import _lib
    text = open(os.path.join(ROOT, "unity", "RaytracingMasterNative.cs")).read()
    body = re.search(r"public struct SvoConfig \{(.*?)\n    \}", text, re.S).group(1)
    names = []
    for decl in re.findall(r"public (uint|int|float) ([^;]+);", body):
        names += [n.strip() for n in decl[1].split(",")]
    snake = [re.sub(r"([A-Z])", lambda m: "_" + m.group(1).lower(), n) for n in names]
    assert snake == ["size", "version"] + [n for n, _ in _lib.CONFIG_FIELDS]
