"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer and under
ThreadSanitizer (its renderer is multithreaded), driven from a plain C process
(tests/sanitize_driver.c): the reference's Text SVO in both stack modes, with and
without shadow rays, two cameras.  The sanitized runs must report nothing and
produce the same bytes as the regular oracle build."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from raytracingtest_amd.camera import main_camera, main_light, overview_camera
from tests.conftest import ROOT

GCC = shutil.which("gcc")
SAN = {
    "asan_ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
    "tsan": ["-fsanitize=thread"],
}


@pytest.fixture(scope="module")
def drivers(tmp_path_factory):
    if GCC is None:
        pytest.skip("gcc not available")
    d = tmp_path_factory.mktemp("san")
    out = {}
    for name, flags in SAN.items():
        exe = str(d / f"drv_{name}")
        cmd = [GCC, "-O1", "-g", "-std=c11", "-ffp-contract=off", "-fno-fast-math", "-pthread", *flags,
               "-I", os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests", "sanitize_driver.c"),
               os.path.join(ROOT, "oracle", "svo_oracle.c"), "-lm", "-o", exe]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            pytest.skip(f"{name} toolchain unavailable: {r.stderr[-400:]}")
        out[name] = exe
    return out


def _input(path, svo, cam, w, h, mode, oracle_mod):
    c2w, inv_proj = cam.uniforms(w, h)
    ocam = oracle_mod.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
    desc = np.asarray(svo.childDescriptors, np.int32)
    att = np.asarray(svo.attachments, np.uint32)
    with open(path, "wb") as f:
        f.write(np.array([len(desc)], np.uint32).tobytes())
        f.write(np.array([w, h, mode, 4], np.int32).tobytes())
        f.write(bytes(ocam))
        f.write(desc.tobytes())
        f.write(att.tobytes())
    return ocam


@pytest.mark.parametrize("san", sorted(SAN))
@pytest.mark.parametrize("mode", [0, 1, 0x100, 0x101])
@pytest.mark.parametrize("camera_name", ["main", "overview"])
def test_oracle_clean_under_sanitizers(drivers, tmp_path, oracle_mod, text_svo, san, mode, camera_name):
    w, h = 96, 64
    cam = main_camera() if camera_name == "main" else overview_camera()
    ocam = _input(tmp_path / "in.bin", text_svo, cam, w, h, mode, oracle_mod)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([drivers[san], str(tmp_path / "in.bin"), str(tmp_path / "out.bin")], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode == 0 and "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-2000:]
    raw = (tmp_path / "out.bin").read_bytes()
    n = w * h
    ref_hits, ref_rgba, _ = oracle_mod.render(oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments),
                                              ocam, w, h, mode)
    assert raw[:24 * n] == ref_hits.tobytes()
    assert raw[24 * n:] == np.asarray(ref_rgba, np.float32).tobytes()
