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
    assert native.svo_abi_version() == _lib.ABI_VERSION == 9
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
