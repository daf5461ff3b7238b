"""GPU parity: the HIP path through the C-ABI vs the CPU oracle, same inputs.

Bar (BASELINE.json north_star): hit voxel (parent, hit_idx, hit_scale, flags)
bit-exact; t and normal within 1e-5 relative -- asserted bit-exact here since
kernel and oracle share the strict-IEEE op order; RGBA of hit pixels within
rtol 1e-5 (miss colour is the procedural sky stand-in, also compared)."""
import re

import numpy as np
import pytest

from raytracingtest_amd import HIT_DTYPE, RaytracingMaster, SVOData, SvoError, band_rows
from raytracingtest_amd.builder import build_from_leaves, build_menger
from raytracingtest_amd.camera import Camera, look_rotation, main_camera, main_light, overview_camera

pytestmark = pytest.mark.gpu

RTOL = 1e-5


@pytest.fixture(scope="module")
def rm():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    m = RaytracingMaster(device=0, capacity_nodes=1 << 22)
    yield m
    m.close()


def _oracle_render(oracle_mod, svo, camera, w, h, mode=0, off=(0.5, 0.5), nodes=False, shadows=False):
    c2w, inv_proj = camera.uniforms(w, h)
    cam = oracle_mod.make_camera(c2w, inv_proj, off, main_light())
    if nodes or svo.format == 2:
        osvo = oracle_mod.OracleSVO(nodes=svo.to_v2(), attachments=svo.attachments)
    else:
        osvo = oracle_mod.OracleSVO(svo.childDescriptors, svo.attachments)
    return oracle_mod.render(osvo, cam, w, h, mode | (oracle_mod.SHADOW_RAYS if shadows else 0))


def _compare(got_hits, got_rgba, ref_hits, ref_rgba):
    g = got_hits.reshape(-1)
    for f in ("parent", "hit_idx", "hit_scale", "flags"):
        bad = np.flatnonzero(g[f] != ref_hits[f])
        assert len(bad) == 0, f"{f} differs at {len(bad)} pixels, first {bad[:5]}"
    for f in ("t", "nx", "ny", "nz"):
        a = g[f].astype(np.float64)
        b = ref_hits[f].astype(np.float64)
        fin = np.isfinite(b)
        assert np.array_equal(np.isfinite(a), fin)
        np.testing.assert_allclose(a[fin], b[fin], rtol=RTOL, atol=0)
    assert g.tobytes() == ref_hits.tobytes(), "hit records not bit-identical"
    if got_rgba is not None:
        np.testing.assert_allclose(got_rgba.reshape(-1, 4), ref_rgba, rtol=RTOL, atol=1e-7)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("camera_name", ["main", "overview"])
def test_text_fixture_parity(rm, oracle_mod, text_svo, mode, camera_name):
    cam = main_camera() if camera_name == "main" else overview_camera()
    w, h = 256, 256   # config C1
    rm.SetSVOBuffer(text_svo)
    rm.UpdateShaderParameters(cam, w, h)
    rgba, hits = rm.Render(w, h, stack_mode=mode)
    ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, text_svo, cam, w, h, mode)
    assert np.count_nonzero(ref_hits["flags"] & 1) > 1000
    _compare(hits, rgba, ref_hits, ref_rgba)


def test_v1_and_v2_uploads_identical(rm, text_svo):
    cam = overview_camera()
    rm.SetSVOBuffer(text_svo)
    rm.UpdateShaderParameters(cam, 320, 200)
    r1, h1 = rm.Render(320, 200)
    rm.SetSVOBuffer(text_svo.as_v2())
    r2, h2 = rm.Render(320, 200)
    assert h1.tobytes() == h2.tobytes() and r1.tobytes() == r2.tobytes()


def test_full_hd_text_fixture(rm, oracle_mod, text_svo):
    cam = overview_camera()
    w, h = 1920, 1080
    rm.SetSVOBuffer(text_svo)
    rm.UpdateShaderParameters(cam, w, h)
    rgba, hits = rm.Render(w, h)
    ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, text_svo, cam, w, h)
    _compare(hits, rgba, ref_hits, ref_rgba)


def test_menger_depth8_parity_and_fetch_counts(rm, oracle_mod):
    torch = pytest.importorskip("torch")
    svo = build_menger(8)
    assert svo.format == 2   # relative pointers overflow 16 bits at 256^3
    cam = overview_camera()
    w, h = 480, 270
    rm.SetSVOBuffer(svo)
    rm.UpdateShaderParameters(cam, w, h)
    rgba, hits = rm.Render(w, h)
    ref_hits, ref_rgba, ref_fetch = _oracle_render(oracle_mod, svo, cam, w, h)
    _compare(hits, rgba, ref_hits, ref_rgba)
    fetch = torch.zeros(w * h, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()   # the fill (torch's stream) before the plugin's own stream writes
    rm.count_fetches_device(w, h, fetch.data_ptr())
    rm.synchronize()
    assert np.array_equal(fetch.cpu().numpy().view(np.uint32), ref_fetch)


def test_band_split_reassembles_frame(rm, text_svo):
    torch = pytest.importorskip("torch")
    cam = overview_camera()
    w, h = 200, 150
    rm.SetSVOBuffer(text_svo)
    rm.UpdateShaderParameters(cam, w, h)
    _, full = rm.Render(w, h)
    out = np.zeros((h, w), full.dtype)
    for rank in range(3):
        band = (8, rank, 3)
        ys = band_rows(h, band)
        buf = torch.zeros(len(ys) * w * 24, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        rm.render_device(w, h, hits_ptr=buf.data_ptr(), band=band)
        rm.synchronize()
        out[ys] = buf.cpu().numpy().view(full.dtype).reshape(len(ys), w)
    assert out.tobytes() == full.tobytes()


def test_jittered_pixel_offset_parity(rm, oracle_mod, text_svo):
    from raytracingtest_amd.camera import jitter_offsets
    cam = main_camera()
    w, h = 128, 96
    rm.SetSVOBuffer(text_svo)
    for off in jitter_offsets(3):
        rm.UpdateShaderParameters(cam, w, h, pixel_offset=tuple(off))
        rgba, hits = rm.Render(w, h)
        ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, text_svo, cam, w, h, off=tuple(off))
        _compare(hits, rgba, ref_hits, ref_rgba)


def test_random_trees_parity(rm, oracle_mod):
    rng = np.random.default_rng(7)
    for depth, n in ((3, 30), (7, 4000), (9, 60000)):
        xyz = np.unique(rng.integers(0, 1 << depth, (n, 3)), axis=0)
        nrm = rng.normal(size=(len(xyz), 3)).astype(np.float32)
        svo = build_from_leaves(depth, xyz, nrm)
        eye = rng.uniform(-30, 30, 3)
        cam = Camera(position=tuple(eye), rotation=look_rotation(-eye + rng.uniform(-5, 5, 3)))
        w, h = 160, 120
        rm.SetSVOBuffer(svo)
        rm.UpdateShaderParameters(cam, w, h)
        for mode in (0, 1):
            rgba, hits = rm.Render(w, h, stack_mode=mode)
            ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, svo, cam, w, h, mode)
            _compare(hits, rgba, ref_hits, ref_rgba)


def test_camera_inside_solid_and_axis_aligned(rm, oracle_mod, text_svo):
    # camera looking exactly down an axis: zero direction components on the centre row/column
    cam = Camera(position=(0.0, 0.0, -40.0), rotation=np.eye(3))
    w, h = 65, 65   # odd size: the centre pixel ray is exactly +z
    rm.SetSVOBuffer(text_svo)
    rm.UpdateShaderParameters(cam, w, h)
    rgba, hits = rm.Render(w, h)
    ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, text_svo, cam, w, h)
    _compare(hits, rgba, ref_hits, ref_rgba)


def test_sub_svo_offset_upload(rm, oracle_mod, text_svo):
    """SetSVOBuffer(data, offset) (RaytracingMaster.cs:118-135): a second pool at a
    descriptor offset; attachments land at 2*offset (documented deviation)."""
    cam = overview_camera()
    w, h = 96, 96
    m = RaytracingMaster(device=0, capacity_nodes=1 << 16)
    try:
        m.SetSVOBuffer(text_svo, offset=0)
        m.SetSVOBuffer(text_svo, offset=10000)
        m.UpdateShaderParameters(cam, w, h)
        rgba, hits = m.Render(w, h)
        ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, text_svo, cam, w, h)
        _compare(hits, rgba, ref_hits, ref_rgba)
        assert m.info()["n_nodes"] == 10000 + len(text_svo)
    finally:
        m.close()


def test_errors_are_loud(rm):
    m = RaytracingMaster(device=0, capacity_nodes=64)
    try:
        with pytest.raises(SvoError):
            m.Render(8, 8)                       # no pool uploaded
        bad = SVOData(childDescriptors=np.array([(100 << 16) | 0x0101], np.int32))
        with pytest.raises(SvoError):
            m.SetSVOBuffer(bad)                  # child pointer outside the capacity
        with pytest.raises(SvoError):
            m.SetSVOBuffer(build_from_leaves(4, np.argwhere(np.ones((16, 16, 16))), np.ones((4096, 3), np.float32)))
    finally:
        m.close()


@pytest.mark.parametrize("cfg", [
    {"xcd_strips": 0}, {"tile_order": 0}, {"issue_priority": 0}, {"fetch_all": 0},
    {"fetch_all": 1}, {"order_every": 1}, {"shadow_order": 0, "shadow_form": 1},
    {"shadow_form": 2}, {"loop_form": 1}, {"loop_form": 0}, {"lat_ratio": 1000.0}])
def test_runtime_switches_identical(oracle_mod, cfg):
    """Every surviving placement / loop-form switch of svo_config (svo_set_config; the
    loop forms and block shapes measured slower in round 1 were removed) gives
    the oracle's frame, over repeated (cost-ordered) launches, with and without
    shadow rays."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    svo = build_menger(7)
    cam = overview_camera()
    w, h = 520, 264
    m = RaytracingMaster(device=0, capacity_nodes=len(svo), config=cfg)
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        for shadows in (False, True):
            ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, svo, cam, w, h, 0, shadows=shadows)
            m.SetShadowRays(shadows)
            for _ in range(3):
                rgba, hits = m.Render(w, h)
                _compare(hits, rgba, ref_hits, ref_rgba)
    finally:
        m.close()


@pytest.mark.parametrize("lat", [0, 1])
def test_degenerate_frame_sizes(oracle_mod, lat):
    """Frames far from the 8x8 tile grid (one pixel, one row, one column, partial
    tiles on both edges) in both loop forms, with and without the fused shadow
    rays, over repeated (cost-ordered) launches: every record equals the oracle's.
    A zero-sized frame is an argument error, not an empty launch."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    svo = build_menger(7)
    m = RaytracingMaster(device=0, capacity_nodes=len(svo), config={"loop_form": lat})
    try:
        m.SetSVOBuffer(svo)
        for cam in (main_camera(), overview_camera()):
            for w, h in ((1, 1), (1, 41), (41, 1), (7, 9), (9, 7), (8, 8), (17, 3), (257, 129)):
                m.UpdateShaderParameters(cam, w, h)
                for shadows in (False, True):
                    ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, svo, cam, w, h, 0, shadows=shadows)
                    m.SetShadowRays(shadows)
                    for _ in range(2):
                        rgba, hits = m.Render(w, h)
                        _compare(hits, rgba, ref_hits, ref_rgba)
        m.SetShadowRays(False)
        for w, h in ((0, 8), (8, 0)):
            with pytest.raises(SvoError):
                m.Render(w, h)
        buf = torch.zeros(64 * 24, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        for w, h in ((-1, 8), (8, -1)):
            with pytest.raises(SvoError):
                m.render_device(w, h, hits_ptr=buf.data_ptr())
    finally:
        m.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_shadow_rays_parity(rm, oracle_mod, mode):
    """C3's '+1 shadow ray' pass: occlusion flag and black
    Result identical to the oracle, on the 256^3 Menger and random terrain."""
    svo = build_menger(8)
    cam = overview_camera()
    w, h = 400, 240
    rm.SetSVOBuffer(svo)
    rm.UpdateShaderParameters(cam, w, h)
    rm.SetShadowRays(True)
    try:
        rgba, hits = rm.Render(w, h, stack_mode=mode)
    finally:
        rm.SetShadowRays(False)
    ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, svo, cam, w, h, mode, shadows=True)
    n_sh = int(np.count_nonzero(ref_hits["flags"] & 8))
    assert 0 < n_sh < np.count_nonzero(ref_hits["flags"] & 1)
    _compare(hits, rgba, ref_hits, ref_rgba)


@pytest.mark.parametrize("form", ["two_pass", "fused", "compact"])
def test_shadow_pass_forms_identical(oracle_mod, form):
    """The shadow rays as a second cost-ordered launch over the tiles
    (shadow_form 1), fused into the primary launch (0, the default), and as a second
    launch over the compacted hit list (2: ballot masks, prefix
    sum, dense waves of 64 hits) give the oracle's frame, over repeated launches
    (the dispatch order is rebuilt from recorded costs) and with RGBA only."""
    svo = build_menger(8)
    cam = overview_camera()
    w, h = 480, 272
    ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, svo, cam, w, h, 0, shadows=True)
    form_id = {"fused": 0, "two_pass": 1, "compact": 2}[form]
    m = RaytracingMaster(device=0, capacity_nodes=len(svo), config={"shadow_form": form_id})
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        m.SetShadowRays(True)
        for _ in range(10):
            rgba, hits = m.Render(w, h)
            _compare(hits, rgba, ref_hits, ref_rgba)
        rgba, _ = m.Render(w, h, want_hits=False)     # shadows without a caller hit buffer
        np.testing.assert_allclose(rgba.reshape(-1, 4), ref_rgba, rtol=RTOL, atol=1e-7)
    finally:
        m.close()


def test_accumulate_matches_oracle(rm, oracle_mod):
    """svo_accumulate (AddShader blend) == the C restatement, bit for bit, over a
    sequence of samples; currentSample advances per blit and resets when the
    camera transform changes (RaytracingMaster.cs:44-47,70-73)."""
    import torch
    rng = np.random.default_rng(11)
    n_px = 1000 * 37 + 3                      # not a multiple of the grid stride
    acc_h = rng.random((n_px, 4), dtype=np.float32)
    acc_d = torch.from_numpy(acc_h.copy()).cuda()
    rm.UpdateShaderParameters(overview_camera(), 64, 64)
    assert rm.currentSample == 0
    for n in range(5):
        smp_h = rng.random((n_px, 4), dtype=np.float32)
        smp_d = torch.from_numpy(smp_h).cuda()
        rm.accumulate_device(acc_d.data_ptr(), smp_d.data_ptr(), n_px)
        oracle_mod.accumulate(acc_h, smp_h, n)
    rm.synchronize()
    torch.cuda.synchronize()
    assert rm.currentSample == 5
    assert acc_d.cpu().numpy().tobytes() == acc_h.tobytes()
    smp_d = torch.from_numpy(rng.random((n_px, 4), dtype=np.float32)).cuda()
    rm.accumulate_device(acc_d.data_ptr(), smp_d.data_ptr(), n_px, sample=1000)
    oracle_mod.accumulate(acc_h, smp_d.cpu().numpy(), 1000)
    rm.synchronize()
    assert acc_d.cpu().numpy().tobytes() == acc_h.tobytes()
    rm.UpdateShaderParameters(main_camera(), 64, 64)   # camera moved -> restart
    assert rm.currentSample == 0
    with pytest.raises(SvoError):
        rm.accumulate_device(acc_d.data_ptr() + 4, smp_d.data_ptr(), n_px)


def test_ordered_dispatch_repeat_renders_identical(rm, oracle_mod):
    """Launches after the first dispatch tiles by recorded cost (heaviest class
    first, interleaved XCD column strips, refreshed every 8th launch): placement
    only, so every frame stays bit-identical to the oracle."""
    svo = build_menger(8)
    cam = overview_camera()
    w, h = 960, 544
    rm.SetSVOBuffer(svo)
    rm.UpdateShaderParameters(cam, w, h)
    ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, svo, cam, w, h)
    for _ in range(10):
        rgba, hits = rm.Render(w, h)
        _compare(hits, rgba, ref_hits, ref_rgba)


def _rounded_parent_pool(base):
    """Depth-3 V2 pool: root -> 8 interior children at base..base+7 -> 64 leaf
    parents (indices 1..64) with one leaf each.  With base = 2^24 - 4 the
    children sit at 2^24 - 4 .. 2^24 + 3, so the HLSL stack round trip
    (int2 <- float2((int)parent, ...), NVIDIASVO.compute:98) turns 2^24 + 1 into
    2^24 (another node) and 2^24 + 3 into 2^24 + 4 == the pool size."""
    n = base + 8
    nodes = np.zeros(n, np.uint64)
    nodes[0] = (np.uint64(base) << np.uint64(32)) | np.uint64(0xFFFF)
    for k in range(8):
        nodes[base + k] = (np.uint64(1 + 8 * k) << np.uint64(32)) | np.uint64(0xFFFF)
    for g in range(1, 65):
        nodes[g] = np.uint64((1 << ((g * 5) % 8)) << 8)      # one leaf child, no non-leaf ones
    return SVOData(nodes=nodes)


def test_out_of_range_rounded_parent_reads_zero(oracle_mod):
    """A pool above 2^24 nodes traced with the HLSL stack: a POP may restore a
    rounded parent index beyond the pool; kernel and oracle both read it as 0
    (an out-of-range StructuredBuffer element) -- bit-identical frames, and
    different from the same tree laid out below 2^24 (so the path is exercised)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    big = _rounded_parent_pool((1 << 24) - 4)
    small = _rounded_parent_pool(65)
    cam = overview_camera()
    w, h = 192, 128
    frames = {}
    for name, svo in (("big", big), ("small", small)):
        m = RaytracingMaster(device=0, capacity_nodes=len(svo))
        try:
            m.SetSVOBuffer(svo)
            m.UpdateShaderParameters(cam, w, h)
            rgba, hits = m.Render(w, h, stack_mode=0)
        finally:
            m.close()
        ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, svo, cam, w, h, mode=0)
        _compare(hits, rgba, ref_hits, ref_rgba)
        frames[name] = hits.reshape(-1)
    hit_big = (frames["big"]["flags"] & 1) != 0
    hit_small = (frames["small"]["flags"] & 1) != 0
    assert hit_small.sum() > 0
    assert np.count_nonzero(hit_big != hit_small) > 0, "no ray went through a rounded parent"


def test_kernel_timing_counts_primary_launches(rm, text_svo):
    """SVO_OPT_KERNEL_TIMING brackets the primary-ray kernel of every launch
    (not the shadow pass); svo_kernel_time returns the mean and forgets them."""
    import torch
    w, h = 256, 128
    rm.SetSVOBuffer(text_svo)
    rm.UpdateShaderParameters(overview_camera(), w, h)
    hits = torch.empty(w * h * 24, dtype=torch.uint8, device="cuda")
    rm.set_kernel_timing(True)
    try:
        rm.kernel_time()
        for _ in range(3):
            rm.render_device(w, h, hits_ptr=hits.data_ptr())
        rm.SetShadowRays(True)
        rm.render_device(w, h, hits_ptr=hits.data_ptr())
        rm.SetShadowRays(False)
        ms, n = rm.kernel_time()
        assert n == 4 and ms > 0.0
        assert rm.kernel_time() == (0.0, 0)
    finally:
        rm.set_kernel_timing(False)
    rm.render_device(w, h, hits_ptr=hits.data_ptr())
    rm.synchronize()
    assert rm.kernel_time() == (0.0, 0)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("camera_name", ["main", "overview"])
def test_c1_golden_frames(rm, text_svo, mode, camera_name):
    """Config C1 (Text SVO, 256x256) on the GPU against the committed golden
    frames (tests/golden/make_c1_golden.py), without running the oracle."""
    import os
    from tests.conftest import GOLDEN
    z = np.load(os.path.join(GOLDEN, "c1_text_frames.npz"))
    key = f"{camera_name}_{'hlsl' if mode == 0 else 'exact'}"
    ref_hits = np.frombuffer(z[key + "_hits"].tobytes(), HIT_DTYPE)
    rm.SetSVOBuffer(text_svo)
    rm.UpdateShaderParameters(main_camera() if camera_name == "main" else overview_camera(), 256, 256)
    rgba, hits = rm.Render(256, 256, stack_mode=mode)
    _compare(hits, rgba, ref_hits, z[camera_name + "_rgba"].reshape(-1, 4))


@pytest.mark.parametrize("stack_mode", [0, 1])
def test_loop_forms_identical_on_a_split_band(oracle_mod, stack_mode):
    """The two loop forms (lean; latency: the node kept in the stack entry, the next node
    loaded mid-trip) and the automatic choice between them (the order kernel's cost stats,
    svo_rt.hip launch) give the oracle's records on a strong-split band of a depth-9 terrain
    pool -- the launch size where the automatic choice switches forms -- over repeated
    launches, both stack modes."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from raytracingtest_amd.native_builder import build_sampler_svo
    svo = build_sampler_svo(4, 10)
    cam = overview_camera()
    w, h = 1024, 576
    band = (8, 1, 4)
    ys = band_rows(h, band)
    ref_hits, ref_rgba, _ = _oracle_render(oracle_mod, svo, cam, w, h, stack_mode)
    ref = ref_hits.reshape(h, w)[ys]
    for lat in (0, 1, -1):   # svo_config.loop_form: lean, latency, automatic
        m = RaytracingMaster(device=0, capacity_nodes=len(svo), config={"loop_form": lat})
        try:
            m.SetSVOBuffer(svo)
            m.UpdateShaderParameters(cam, w, h)
            buf = torch.empty(len(ys) * w * 24, dtype=torch.uint8, device="cuda")
            for _ in range(6):   # the order (and its stats) exist from the second launch on
                m.render_device(w, h, hits_ptr=buf.data_ptr(), band=band, stack_mode=stack_mode)
                m.synchronize()
                got = buf.cpu().numpy().view(ref.dtype).reshape(len(ys), w)
                assert got.tobytes() == ref.tobytes(), f"loop_form={lat}"
        finally:
            m.close()


_DECISION = re.compile(r"svo lat: view (\d+) T \d+ M \d+ slots \d+ ratio ([0-9.]+) bound ([0-9.]+) "
                       r"thin ([0-9.]+) beam (\d) -> (\w+)( thin)?")


def _pose_decisions(monkeypatch, capfd, config, plan):
    """Render the C3 frame at each pose of `plan` as a burst of 12 launches with no host sync (the
    host runs ahead of the GPU) and return, per pose, the decisions the library's SVO_DEBUG trace
    printed for that pose's view: (ratio, bound, thin_bound, beam, form, thin)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    monkeypatch.setenv("SVO_DEBUG", "1")   # diagnostics only: the decision trace (read at svo_create)
    svo = build_sampler_svo(4, 11)   # config C3's pool
    w, h = 1920, 1080
    m = RaytracingMaster(device=0, capacity_nodes=len(svo), config=config)
    out = []
    try:
        m.SetSVOBuffer(svo)
        buf = torch.empty(w * h * 24, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        for view, pose in enumerate(plan, start=1):
            capfd.readouterr()
            m.UpdateShaderParameters(CAMERAS[pose](), w, h)
            for _ in range(12):
                m.render_device(w, h, hits_ptr=buf.data_ptr(), stack_mode=0)
            m.synchronize()
            err = capfd.readouterr().err
            found = _DECISION.findall(err)
            mine = [(float(r), float(b), float(tb), int(be), f, bool(th)) for v, r, b, tb, be, f, th in found
                    if int(v) == view]
            assert mine, f"no decision from view {view} ({pose}): {err[-2000:]}"
            assert all(int(v) >= view - 1 for v, *_ in found), f"{pose}: stale decisions {found}"
            out.append((pose, mine))
    finally:
        m.close()
    return out


def test_loop_form_choice_follows_the_pose(monkeypatch, capfd):
    """The automatic loop form (svo_rt.hip launch) is decided from the dispatch-order build
    of the CURRENT camera view: across jumps between unrelated poses of the C3 frame, each
    submitted as a burst of launches with no host sync (the host runs ahead of the GPU),
    every decision taken at a pose uses that pose's own costs -- the sky-heavy overview the
    latency form, the flyover and Main poses the lean loop (costs of the walk from
    the cube entry, beam 0 -- beam starts shorten every wave but the heaviest and make the
    flyover pose latency-bound too).  Reads the library's SVO_DEBUG decision trace."""
    plan = ["flyover", "overview", "main", "overview"]
    want = {"flyover": "lean", "overview": "latency", "main": "lean"}
    for pose, mine in _pose_decisions(monkeypatch, capfd, {"beam": 0}, plan):
        assert all(d[3] == 0 for d in mine)
        assert all(d[4] == want[pose] for d in mine), f"{pose}: {mine}"


def test_class_table_choice_follows_the_pose_with_beam_starts(monkeypatch, capfd):
    """The default launch (beam starts on): the same jumps between the C3 poses, and each view's
    class-table decision (issue-bound table, latency-bound table, or the thin table) is the current
    rule applied to that view's own statistics (svo_rt.hip launch: latency-bound iff the summed
    trips T < bound x slots x heaviest M -- bound = seg_ratio 0.28, x/÷ 1.15 once the geometry has a
    decision -- and thin iff also below seg_thin_ratio 0.083): the trace's ratio, bound and form
    agree.  Beside the rule, the poses far from a boundary take their table: the sky-heavy overview
    (ratio ~0.06) the thin table, the Main.unity pose (~0.49) the issue-bound one."""
    plan = ["flyover", "overview", "main", "overview", "flyover"]
    for pose, mine in _pose_decisions(monkeypatch, capfd, None, plan):
        for ratio, bound, thin_bound, beam, form, thin in mine:
            assert beam == 1
            assert (form == "latency") == (ratio < bound), f"{pose}: {mine}"
            assert thin == (form == "latency" and ratio < thin_bound), f"{pose}: {mine}"
        table = {"latency": "thin" if mine[-1][5] else "latency", "lean": "issue"}[mine[-1][4]]
        if pose == "overview":
            assert table == "thin", f"{pose}: {mine}"
        if pose == "main":
            assert table == "issue", f"{pose}: {mine}"
