"""The C-ABI from a plain C host (examples/render_min.c): no Python, no torch
between the caller and libsvo_rt.so -- the boundary a native engine binds."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(ROOT, "raytracingtest_amd")
SRC = os.path.join(ROOT, "examples", "render_min.c")


def _build(tmp_path):
    if not os.path.exists(os.path.join(LIB_DIR, "libsvo_rt.so")):
        pytest.skip("libsvo_rt.so not built (run __graft_entry__.build())")
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = str(tmp_path / "render_min")
    subprocess.run([cc, "-O2", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), SRC,
                    "-L", LIB_DIR, "-lsvo_rt", "-L/opt/rocm/lib", "-lamdhip64", "-lm",
                    "-Wl,-rpath," + LIB_DIR, "-Wl,-rpath,/opt/rocm/lib", "-o", exe], check=True)
    return exe


def test_c_host_compiles_and_links(tmp_path):
    assert os.path.exists(_build(tmp_path))


@pytest.mark.gpu
def test_c_host_renders(tmp_path):
    exe = _build(tmp_path)
    out = subprocess.run([exe, str(tmp_path / "frame.ppm")], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "render_min: ok" in out.stdout
    assert (tmp_path / "frame.ppm").stat().st_size == len("P6\n64 64\n255\n") + 64 * 64 * 3
