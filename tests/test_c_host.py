"""The C-ABI from a plain C host (examples/render_min.c, examples/build_and_render.c):
no Python, no torch between the caller and libsvo_rt.so / libsvo_build.so -- the
boundary a native engine binds."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(ROOT, "raytracingtest_amd")
SRC = os.path.join(ROOT, "examples", "render_min.c")


def _build(tmp_path, src=SRC, name="render_min", libs=("-lsvo_rt",), extra=()):
    for lib in libs:
        if not os.path.exists(os.path.join(LIB_DIR, "lib" + lib[2:] + ".so")):
            pytest.skip(f"lib{lib[2:]}.so not built (run __graft_entry__.build())")
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = str(tmp_path / name)
    subprocess.run([cc, "-O2", "-std=c99", "-Wall", "-Werror", *extra, "-I", os.path.join(ROOT, "include"), src,
                    "-L", LIB_DIR, *libs, "-L/opt/rocm/lib", "-lamdhip64", "-lm",
                    "-Wl,-rpath," + LIB_DIR, "-Wl,-rpath,/opt/rocm/lib", "-o", exe], check=True)
    return exe


def _build_key_r(tmp_path):
    return _build(tmp_path, os.path.join(ROOT, "examples", "build_and_render.c"), "build_and_render",
                  ("-lsvo_rt", "-lsvo_build"))


def _build_bench(tmp_path):
    if not os.path.exists("/opt/rocm/include/hip/hip_runtime_api.h"):
        pytest.skip("no HIP headers")
    return _build(tmp_path, os.path.join(ROOT, "examples", "bench_native.c"), "bench_native",
                  ("-lsvo_rt", "-lsvo_build"), ("-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"))


def _camera_blob(W, H, name="flyover"):
    import numpy as np
    from raytracingtest_amd.camera import CAMERAS, column_major, main_light
    c2w, inv_proj = CAMERAS[name]().uniforms(W, H)
    blob = np.concatenate([column_major(np.asarray(c2w, np.float32)).reshape(-1),
                           column_major(np.asarray(inv_proj, np.float32)).reshape(-1),
                           np.asarray(main_light(), np.float32)]).astype(np.float32)
    assert blob.size == 36
    return blob.tobytes()


def test_c_host_compiles_and_links(tmp_path):
    assert os.path.exists(_build(tmp_path))


@pytest.mark.gpu
def test_c_host_renders(tmp_path):
    exe = _build(tmp_path)
    out = subprocess.run([exe, str(tmp_path / "frame.ppm")], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "render_min: ok" in out.stdout
    assert (tmp_path / "frame.ppm").stat().st_size == len("P6\n64 64\n255\n") + 64 * 64 * 3


def test_c_bench_host_compiles_and_links(tmp_path):
    assert os.path.exists(_build_bench(tmp_path))


@pytest.mark.gpu
def test_c_bench_host_runs(tmp_path):
    """examples/bench_native.c: the metric's frame (C3 pool, 1920x1080, flyover) timed from a
    plain C process through the C-ABIs alone; a short run here, the full one in profiles/."""
    import json
    exe = _build_bench(tmp_path)
    (tmp_path / "cam.bin").write_bytes(_camera_blob(1920, 1080))
    out = subprocess.run([exe, "4", "11", str(tmp_path / "cam.bin"), "1920", "1080", "20", "5"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["nodes"] == 1569748 and r["stack_mode"] == "hlsl" and r["kernel_launches"] == 20
    assert 0.0 < r["kernel_ms"] <= r["ms_per_step"] * 1.5
    assert r["Mrays_per_s"] > 1000.0


def test_c_host_key_r_compiles_and_links(tmp_path):
    assert os.path.exists(_build_key_r(tmp_path))


@pytest.mark.gpu
def test_c_host_builds_uploads_v2_and_renders(tmp_path, oracle_mod):
    """The reference's key-R path from C (RaytracingMaster.cs:50-52,90-109): the native
    NaiveCreator builds the depth-10 Custom1 pool (C3's, child pointers beyond 16 bits),
    svo_set_buffer_v2 uploads it, svo_get_info picks the stack mode, svo_render traces a
    reduced 480x270 frame from the flyover camera; every hit record equals the oracle's
    on the same pool (built again here, deterministically) and camera."""
    import numpy as np
    from raytracingtest_amd import HIT_DTYPE
    from raytracingtest_amd.camera import CAMERAS, column_major, main_light
    from raytracingtest_amd.native_builder import build_sampler_svo
    exe = _build_key_r(tmp_path)
    W, H = 480, 270
    cam = CAMERAS["flyover"]()
    c2w, inv_proj = cam.uniforms(W, H)
    light = np.asarray(main_light(), np.float32)
    blob = np.concatenate([column_major(np.asarray(c2w, np.float32)).reshape(-1),
                           column_major(np.asarray(inv_proj, np.float32)).reshape(-1), light]).astype(np.float32)
    assert blob.size == 36
    (tmp_path / "cam.bin").write_bytes(blob.tobytes())
    out = subprocess.run([exe, "4", "11", str(tmp_path / "cam.bin"), str(W), str(H), str(tmp_path / "hits.bin"),
                          str(tmp_path / "rgba.bin")], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "v1 pointers overflow" in out.stdout and "stack mode hlsl" in out.stdout, out.stdout
    got = np.frombuffer((tmp_path / "hits.bin").read_bytes(), HIT_DTYPE)
    rgba = np.frombuffer((tmp_path / "rgba.bin").read_bytes(), np.float32).reshape(-1, 4)
    svo = build_sampler_svo(4, 11)
    assert svo.format == 2
    ocam = oracle_mod.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
    osvo = oracle_mod.OracleSVO(nodes=svo.to_v2(), attachments=svo.attachments)
    ref, ref_rgba, _ = oracle_mod.render(osvo, ocam, W, H, 0, want_fetches=False)
    assert np.count_nonzero(ref["flags"] & 1) > 10000
    assert got.tobytes() == ref.tobytes()
    np.testing.assert_allclose(rgba, ref_rgba, rtol=1e-5, atol=1e-7)


def _build_async(tmp_path):
    return _build(tmp_path, os.path.join(ROOT, "examples", "progressive_async.c"), "progressive_async",
                  extra=("-D_POSIX_C_SOURCE=199309L",))


def test_c_host_progressive_async_compiles_and_links(tmp_path):
    assert os.path.exists(_build_async(tmp_path))


@pytest.mark.gpu
@pytest.mark.parametrize("rgb", [False, True])
def test_c_host_progressive_async_frames_match_oracle(tmp_path, oracle_mod, text_svo, rgb):
    """the Unity loop through svo_render_progressive_async from plain C --
    a new jittered _PixelOffset per frame, each call returning the previous frame from the
    plugin's pinned slots -- displays exactly the oracle's accumulation (per-sample render
    + orc_accumulate + orc_pack_rgba8) frame after frame, the last one via
    svo_progressive_last."""
    import json

    import numpy as np
    from raytracingtest_amd.camera import CAMERAS, jitter_offsets, main_light
    exe = _build_async(tmp_path)
    W, H, N = 96, 70, 6
    pool = np.concatenate([np.array([len(text_svo.childDescriptors), len(text_svo.attachments)], np.uint32),
                           text_svo.childDescriptors.view(np.uint32), text_svo.attachments.astype(np.uint32)])
    (tmp_path / "pool.bin").write_bytes(pool.tobytes())
    (tmp_path / "cam.bin").write_bytes(_camera_blob(W, H, "overview"))
    offs = jitter_offsets(N)
    (tmp_path / "offs.bin").write_bytes(offs.astype(np.float32).tobytes())
    out = subprocess.run([exe, str(tmp_path / "pool.bin"), str(tmp_path / "cam.bin"), str(tmp_path / "offs.bin"),
                          str(W), str(H), str(N), str(tmp_path / "frames.bin")] + (["rgb"] if rgb else []),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert json.loads(out.stdout.strip().splitlines()[-1])["frames"] == N
    if rgb:   # SVO_PIXELS_RGB8: the display words without their alpha byte
        px = np.fromfile(tmp_path / "frames.bin", np.uint8).reshape(N, W * H, 3).astype(np.uint32)
        got = px[..., 0] | (px[..., 1] << 8) | (px[..., 2] << 16) | np.uint32(255 << 24)
    else:
        got = np.fromfile(tmp_path / "frames.bin", np.uint32).reshape(N, W * H)
    c2w, inv_proj = CAMERAS["overview"]().uniforms(W, H)
    osvo = oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments)
    acc = np.zeros((W * H, 4), np.float32)
    for k in range(N):
        _, smp, _ = oracle_mod.render(osvo, oracle_mod.make_camera(c2w, inv_proj, tuple(float(v) for v in offs[k]),
                                                                  main_light()), W, H)
        oracle_mod.accumulate(acc, np.ascontiguousarray(smp, np.float32), k)
        assert np.array_equal(got[k], oracle_mod.pack_rgba8(acc)), f"frame {k}"
