"""Pin the CPU oracle: reference fixtures (decode KATs) + independent brute force."""
import os

import numpy as np
import pytest

from raytracingtest_amd.camera import main_camera, main_light, overview_camera
from raytracingtest_amd.svo_data import SVOData
from tests.bruteforce import entry_exit, first_hits, svo_space_ray
from tests.conftest import GOLDEN


def _cam(oracle_mod, camera, w, h, off=(0.5, 0.5)):
    c2w, inv_proj = camera.uniforms(w, h)
    return oracle_mod.make_camera(c2w, inv_proj, off, main_light())


def test_decode_normal_matches_text_dump(oracle_mod, text_fixture):
    """4,977 known answers: Text prints Normalize(decodeRawNormal16(code)) with F1
    (NaiveCreator.cs:573-595 == AttachmentLookup.compute:37-61)."""
    codes = text_fixture["normal_code"]
    printed = text_fixture["normal_f1"]
    bad = 0
    for code, ref in zip(codes, printed):
        n = oracle_mod.decode_normal(int(code)).astype(np.float64)
        n /= np.linalg.norm(n)
        # .NET "F1" rounds half away from zero; allow the tie band
        if np.any(np.abs(n - ref) > 0.05 + 1e-6):
            bad += 1
    assert bad == 0


def test_decode_normal_axis_permutation(oracle_mod):
    # axis bits 0x2000 -> (v, t, u); 0x4000 -> (u, v, t); sign bit -> t = -32768
    assert list(oracle_mod.decode_normal(0x0000)) == [32767.0, 0.0, 0.0]
    assert list(oracle_mod.decode_normal(0x8000)) == [-32768.0, 0.0, 0.0]
    assert list(oracle_mod.decode_normal(0x2000)) == [0.0, 32767.0, 0.0]
    assert list(oracle_mod.decode_normal(0x4000)) == [0.0, 0.0, 32767.0]
    # u = bits 0..12 sign-extended x 8, v = bits 0..5 sign-extended x 1024
    def sext(x, bits):
        return x - (1 << bits) if x & (1 << (bits - 1)) else x
    for code in (0x0FDF, 0x1040, 0x003F, 0x0020, 0x1FFF, 0x0ABC):
        n = oracle_mod.decode_normal(code)
        assert n[1] == sext(code & 0x1FFF, 13) * 8
        assert n[2] == sext(code & 0x3F, 6) * 1024


def test_decode_dxt_color_selects_endpoints(oracle_mod):
    rng = np.random.default_rng(1)
    for _ in range(200):
        a, b = (int(v) for v in rng.integers(0, 1 << 16, 2))
        head = a | (b << 16)
        ca = oracle_mod.decode_dxt_color(head, 0x0, 0)      # choice 0 -> colour A
        cb = oracle_mod.decode_dxt_color(head, 0x1, 0)      # choice 1 -> colour B
        # the reference decode keeps the lower channels' bits below each channel:
        # channel = float32((head << k) mod 2^32) / 2^32 (AttachmentLookup.compute:12-17)
        def chan(h, k):
            return np.float32(np.float32((h << k) & 0xFFFFFFFF) / np.float32(2.0 ** 32))
        np.testing.assert_array_equal(ca, [chan(head, 27), chan(head, 21), chan(head, 16)])
        np.testing.assert_array_equal(cb, [chan(head, 11), chan(head, 5), chan(head, 0)])
        assert abs(ca[0] - (a & 31) / 32) < 1e-9 and abs(ca[1] - ((a >> 5) & 63) / 64) < 1 / 64
        # choices 2/3 blend 2:1 and 1:2
        c2 = oracle_mod.decode_dxt_color(head, 0x2, 0).astype(np.float64)
        np.testing.assert_allclose(c2, (2 * ca + cb) / 3, atol=1e-6)
        # texel index selects its own 2-bit field
        c7 = oracle_mod.decode_dxt_color(head, 0x1 << 14, 7)
        np.testing.assert_array_equal(c7, cb)


def test_camera_ray_center_pixel(oracle_mod):
    cam = _cam(oracle_mod, main_camera(), 256, 256)
    o, d = oracle_mod.camera_ray(cam, 128, 128, 256, 256)   # uv = (0.5/256*2... ) ~ centre
    np.testing.assert_allclose(o, [1, 1, 1], atol=1e-6)
    assert d[2] > 0.99   # identity rotation looks down +z
    assert abs(np.linalg.norm(d) - 1) < 1e-6


_FRAME_RAYS = {}


def _frame_rays(oracle_mod, camera_name, w, h):
    """World-space camera rays of every pixel (the oracle's CreateCameraRay)."""
    key = (camera_name, w, h)
    if key not in _FRAME_RAYS:
        cam = _cam(oracle_mod, main_camera() if camera_name == "main" else overview_camera(), w, h)
        o = np.zeros((h * w, 3), np.float32)
        d = np.zeros((h * w, 3), np.float32)
        for y in range(h):
            for x in range(w):
                o[y * w + x], d[y * w + x] = oracle_mod.camera_ray(cam, x, y, w, h)
        _FRAME_RAYS[key] = (cam, o, d)
    return _FRAME_RAYS[key]


_BRUTE = {}


@pytest.mark.parametrize("stack_mode", [0, 1])
@pytest.mark.parametrize("camera_name", ["main", "overview"])
def test_traversal_matches_bruteforce_full_c1_frame(oracle_mod, text_svo, camera_name, stack_mode):
    """Every ray of the full 256x256 C1 frame (Text SVO, both cameras, both
    stack modes) against the double-precision brute force over all 10,464
    leaves: the oracle's voxel is a first-hit voxel up to ties, its t is the
    voxel's entry distance, its scale the leaf's, and a miss only skips voxels
    the ray grazes."""
    from tests.bruteforce import first_hits_compact
    w = h = 256
    cam, o, d = _frame_rays(oracle_mod, camera_name, w, h)
    hits, _, _ = oracle_mod.render(oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments),
                                   cam, w, h, stack_mode)
    leaves = text_svo.leaf_voxels()
    oo = o.astype(np.float64) / 32.0 + 1.5
    dd = d.astype(np.float64)
    if camera_name not in _BRUTE:
        _BRUTE[camera_name] = first_hits_compact(leaves, oo, dd)
    best_row, best_t, max_ov = _BRUTE[camera_name]
    miss = hits["parent"] == 0xFFFFFFFF
    assert not np.any(max_ov[miss] > 1e-5), "oracle miss where the brute force crosses a voxel"
    assert not np.any(~miss & (best_row < 0) & (max_ov < -1)), "oracle hit where the ray touches no voxel"
    key = {(int(r[0]), int(r[1])): i for i, r in enumerate(leaves)}
    n_hit = 0
    for i in np.flatnonzero(~miss):
        hrec = hits[i]
        row = key[(int(hrec["parent"]), int(hrec["hit_idx"]))]
        nz = np.abs(dd[i])[np.abs(dd[i]) > 0]
        tol = 1e-6 * (1.0 + 3.0 / nz.min())
        t_in, t_out = entry_exit(leaves[row], oo[i], dd[i])
        assert t_in <= t_out + tol, f"ray {i}: oracle voxel not on the ray"
        assert t_in <= best_t[i] + tol, f"ray {i}: oracle voxel enters at {t_in} > {best_t[i]}"
        assert abs(hrec["t"] / 2048.0 - t_in) <= tol
        assert hrec["hit_scale"] == 23 - leaves[row, 2]
        n_hit += 1
    assert n_hit > 2000


@pytest.mark.parametrize("camera_name", ["main", "overview"])
def test_oracle_exact_mode_matches_csharp_raystep(oracle_mod, text_fixture, text_svo, camera_name):
    """Second independent witness of the hot loop: the reference's own C# CPU
    tracer NVIDIAIterativeNaiveTracer.RayStep (NVIDIAIterativeTracer.cs:72-290),
    restated in tests/cs_tracer.py over ABSOLUTE pointers (the Text dump's native
    form), exact stack, popc8 LUT, t_max clamped to 1 (:112).  On the full 256x256
    C1 frames the oracle's EXACT stack mode must give the same voxel (parent,
    hit_idx, scale) and bit-identical t for every ray whose hit lies within
    t_svo <= 1 -- the clamp cannot change any decision before such a hit, since
    t_min only grows and stays <= 1 -- and the C# tracer must miss every other ray."""
    from tests.cs_tracer import descriptors_absolute, ray_step
    w = h = 256
    cam, o, d = _frame_rays(oracle_mod, camera_name, w, h)
    hits, _, _ = oracle_mod.render(oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments),
                                   cam, w, h, oracle_mod.STACK_EXACT)
    z = text_fixture
    svo_cs = descriptors_absolute(z["abs_child_ptr"], z["valid_mask"], z["nonleaf_mask"])
    # the HLSL world -> SVO transform (NVIDIASVO.compute:15-19) feeds the caller-space C# tracer
    o_svo = o * np.float32(1.0 / 32.0) + np.float32(1.5)
    r = ray_step(svo_cs, o_svo, d)
    reach = (hits["parent"] != 0xFFFFFFFF) & (hits["t"] <= np.float32(2048.0))
    assert np.array_equal(r["hit"], reach), f"{np.count_nonzero(r['hit'] != reach)} rays differ in hit/miss"
    assert np.array_equal(r["parent"][reach], hits["parent"][reach].astype(np.int64))
    assert np.array_equal(r["hit_idx"][reach], hits["hit_idx"][reach].astype(np.int32))
    assert np.array_equal(r["scale"][reach], hits["hit_scale"][reach].astype(np.int32))
    t_cs = (r["t_min"][reach] * np.float32(2048.0)).astype(np.float32)
    assert t_cs.tobytes() == hits["t"][reach].astype(np.float32).tobytes()
    assert np.count_nonzero(reach) > 2000


def test_decode_dxt_color_worked_example(oracle_mod):
    """The reference's worked attachment example (NaiveCreator.cs:260-292, printed
    by TestDecompressAttachment :296-345 with Vector3's F1 format): NodeAColor
    0100110001111100 and NodeBColor 1110011011101011 decode through
    decodeDXTColor to C0 (0.5, 0.8, 0.7) and C1..C7 (0.9, 0.6, 0.3).  The printed
    ColorChoices line is stale (all ones would make every child C0's colour);
    the printed children need child 0's choice = 3 and the others 0, i.e.
    bits = 3.  The raw attachment string pins the 64-bit layout A | B << 16 |
    choices << 32 | normal << 48 (GetAttachment :247)."""
    a, b = 0b0100110001111100, 0b1110011011101011
    raw = "1111111111111111111111111111111111100110111010110100110001111100"
    v = int(raw, 2)
    assert v & 0xFFFF == a and (v >> 16) & 0xFFFF == b and (v >> 32) & 0xFFFF == 0xFFFF
    head = a | (b << 16)
    want = [(0.5, 0.8, 0.7)] + [(0.9, 0.6, 0.3)] * 7
    for texel, w in enumerate(want):
        got = oracle_mod.decode_dxt_color(head, 3, texel).astype(np.float64)
        assert np.all(np.abs(got - w) <= 0.05 + 1e-6), (texel, got)
    # "Partially Decompressed" (DecompressColor, :357-362): R in the low 5 bits
    def decompress(c):
        return np.array([(c & 31) / 31.0, ((c >> 5) & 63) / 63.0, (c >> 11) / 31.0])
    assert np.all(np.abs(decompress(a) - (0.9, 0.6, 0.3)) <= 0.05 + 1e-6)
    assert np.all(np.abs(decompress(b) - (0.4, 0.9, 0.9)) <= 0.05 + 1e-6)


def test_v1_and_v2_pools_identical(oracle_mod, text_svo):
    cam = _cam(oracle_mod, overview_camera(), 96, 64)
    a = oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments)
    b = oracle_mod.OracleSVO(nodes=text_svo.to_v2(), attachments=text_svo.attachments)
    ha, ra, fa = oracle_mod.render(a, cam, 96, 64)
    hb, rb, fb = oracle_mod.render(b, cam, 96, 64)
    assert ha.tobytes() == hb.tobytes()
    assert ra.tobytes() == rb.tobytes()
    assert np.array_equal(fa, fb)
    # the oracle's own v1->v2 conversion equals the product-side one
    assert np.array_equal(oracle_mod.v1_to_v2(text_svo.childDescriptors), text_svo.to_v2())


def test_axis_aligned_and_degenerate_rays(oracle_mod, text_svo):
    """Zero direction components give 1/-0 = -inf and NaN t-values that min/max
    drop (NVIDIASVO.compute:21-32, the epsilon clamp is commented out).  The
    NaN centre tests then always pick the low child along that axis, so exactly
    axis-aligned rays follow the reference's (non-geometric) semantics: the
    oracle must terminate with finite t and report voxels of the low half only.
    Nearly axis-aligned rays (|d_i| = 1e-3) must agree with the brute force."""
    osvo = oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments)
    leaves = text_svo.leaf_voxels()
    key = {(int(r[0]), int(r[1])): i for i, r in enumerate(leaves)}
    for axis in range(3):
        for sgn in (1.0, -1.0):
            for off in (-0.3, 0.0, 0.37, 7.9):
                for tiny in (0.0, 1e-3):
                    d = np.full(3, tiny, np.float32)
                    d[axis] = sgn
                    d /= np.linalg.norm(d)
                    o = np.full(3, off, np.float32)
                    o[axis] = -40.0 * sgn
                    hrec, _, f, it = oracle_mod.intersect(osvo, o, d)
                    assert it < 65536 and hrec["flags"] & 2 == 0
                    if hrec["parent"] != 0xFFFFFFFF:
                        assert np.isfinite(hrec["t"]) and hrec["t"] > 0
                    if tiny == 0.0:
                        continue
                    oo, dd = svo_space_ray(o, d)
                    br, bt, te, ov = first_hits(leaves, oo[None], dd[None])
                    if hrec["parent"] == 0xFFFFFFFF:
                        assert not np.any(ov[0] > 1e-5)
                    else:
                        row = key[(int(hrec["parent"]), int(hrec["hit_idx"]))]
                        t_in, t_out = entry_exit(leaves[row], oo, dd)
                        assert t_in <= t_out + 1e-2 and t_in <= bt[0] + 1e-2


def test_rays_missing_the_cube(oracle_mod, text_svo):
    osvo = oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments)
    for o, d in [((100, 100, 100), (1, 0, 0)), ((0, 40, 0), (0, 1, 0)), ((-40, 0, 0), (-1, 0.1, 0))]:
        d = np.asarray(d, np.float32) / np.linalg.norm(d)
        h, alb, f, it = oracle_mod.intersect(osvo, np.float32(o), d)
        assert h["parent"] == 0xFFFFFFFF and np.isinf(h["t"]) and h["flags"] == 0


def test_empty_pool_is_all_miss(oracle_mod):
    empty = SVOData(childDescriptors=np.zeros(1, np.int32))
    osvo = oracle_mod.OracleSVO(empty.childDescriptors, empty.attachments)
    cam = _cam(oracle_mod, overview_camera(), 32, 32)
    hits, rgba, fet = oracle_mod.render(osvo, cam, 32, 32)
    assert np.all(hits["parent"] == 0xFFFFFFFF)
    assert np.all(rgba[:, 3] == 1.0)


def test_hlsl_stack_roundtrip_rarely_changes_hits(oracle_mod, text_svo):
    """HLSL mode rounds the stacked t_max to 24 significant bits of its bit
    pattern; EXACT keeps it.  Hits may only differ in rare grazing cases."""
    cam = _cam(oracle_mod, overview_camera(), 128, 128)
    osvo = oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments)
    h0, _, _ = oracle_mod.render(osvo, cam, 128, 128, 0)
    h1, _, _ = oracle_mod.render(osvo, cam, 128, 128, 1)
    diff = np.count_nonzero((h0["parent"] != h1["parent"]) | (h0["hit_idx"] != h1["hit_idx"]))
    assert diff <= len(h0) // 1000


def test_accumulate_known_answers(oracle_mod):
    """AddShader blend (AddShader.shader:10,44-47): sample 0 replaces the frame,
    sample n weights the new frame 1/(n+1); a constant stream stays constant and
    n frames average (f32 formula, written out here in numpy)."""
    rng = np.random.default_rng(3)
    dst = rng.random((7, 5, 4), dtype=np.float32)
    src = rng.random((7, 5, 4), dtype=np.float32)
    out = oracle_mod.accumulate(dst.copy(), src, 0)
    assert np.array_equal(out[..., :3], src[..., :3]) and np.all(out[..., 3] == 1.0)
    for n in (1, 2, 7, 1000):
        a = np.float32(1.0) / (np.float32(n) + np.float32(1.0))
        b = np.float32(1.0) - a
        want = dst.copy()
        want[..., :3] = src[..., :3] * a + dst[..., :3] * b
        want[..., 3] = a * a + dst[..., 3] * b
        got = oracle_mod.accumulate(dst.copy(), src, n)
        assert got.tobytes() == want.tobytes(), n
    acc = np.zeros((3, 3, 4), np.float32)
    frames = rng.random((6, 3, 3, 4), dtype=np.float32)
    for n, f in enumerate(frames):
        oracle_mod.accumulate(acc, np.ascontiguousarray(f), n)
    np.testing.assert_allclose(acc[..., :3], frames[..., :3].mean(0), rtol=1e-5)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("camera_name", ["main", "overview"])
def test_oracle_reproduces_c1_golden_frames(oracle_mod, text_svo, mode, camera_name):
    """The oracle's C1 frames (Text SVO, 256x256) are bit-identical to the committed
    golden vectors (tests/golden/make_c1_golden.py): a compiler, flag or code change
    that moves any bit of a hit record or Result pixel is caught here."""
    from raytracingtest_amd.camera import main_camera, main_light, overview_camera
    z = np.load(os.path.join(GOLDEN, "c1_text_frames.npz"))
    key = f"{camera_name}_{'hlsl' if mode == 0 else 'exact'}"
    cam = main_camera() if camera_name == "main" else overview_camera()
    c2w, inv_proj = cam.uniforms(256, 256)
    ocam = oracle_mod.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
    hits, rgba, _ = oracle_mod.render(oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments),
                                      ocam, 256, 256, mode)
    assert hits.tobytes() == z[key + "_hits"].tobytes()
    assert rgba.astype(np.float32).tobytes() == z[camera_name + "_rgba"].tobytes()


def test_shadow_iteration_counts_diagnostic(oracle_mod, text_svo):
    """COUNT_SHADOW_ITERS (the r02 shadow-compaction model): the per-pixel output counts the
    shadow ray's loop iterations, 0 exactly where no shadow ray is traced; the
    records are the same as without the diagnostic."""
    from raytracingtest_amd.camera import main_camera, main_light
    w = h = 64
    c2w, inv_proj = main_camera().uniforms(w, h)
    cam = oracle_mod.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
    svo = oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments)
    hits, _, sit = oracle_mod.render(svo, cam, w, h, oracle_mod.SHADOW_RAYS | oracle_mod.COUNT_SHADOW_ITERS)
    ref, _, _ = oracle_mod.render(svo, cam, w, h, oracle_mod.SHADOW_RAYS)
    assert hits.tobytes() == ref.tobytes()
    hit = (hits["flags"] & 1) != 0
    assert hit.any() and np.all(sit[~hit] == 0) and np.all(sit[hit] > 0)
