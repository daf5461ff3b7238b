"""GPU parity of the frame outputs and of the multi-GPU split, through the C-ABI.

* every per-pixel output of svo_render_frame (hit records, Result, display
  RGBA8, compact records, bestHit.position, voxel key) against the oracle,
  bit for bit (NVIDIASVO.compute:158-186, RaytraceCompute.compute:93-127,167);
* the north-star split: a multi-device context (svo_create_multi) with the
  device index repeated -- one MI355X renders every member's bands and the
  display member pulls the payloads exactly as it would over xGMI -- and the
  one-process-per-GPU form (band parts rendered separately, rebuilt by
  svo_assemble_frame), both bit-identical to the oracle's single frame;
* the round-1 advisor cases: launches alternating between two streams, a DAG
  pool whose shared node sits at two depths, a chain of three linked pools.
"""
import numpy as np
import pytest

from raytracingtest_amd import HIT_DTYPE, RaytracingMaster, SvoError, band_rows
from raytracingtest_amd import _lib
from raytracingtest_amd.builder import build_menger
from raytracingtest_amd.camera import CAMERAS, Camera, look_rotation, main_camera, main_light, overview_camera
from raytracingtest_amd.svo_data import SVOData

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    t = pytest.importorskip("torch")
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def _oracle(oracle_mod, svo, cam, w, h, mode=0, off=(0.5, 0.5), shadows=False):
    c2w, inv_proj = cam.uniforms(w, h)
    ocam = oracle_mod.make_camera(c2w, inv_proj, off, main_light())
    osvo = oracle_mod.OracleSVO(nodes=svo.to_v2(), attachments=svo.attachments)
    if shadows:
        hits, rgba, _ = oracle_mod.render(osvo, ocam, w, h, mode | oracle_mod.SHADOW_RAYS)
        return hits, rgba, None, None
    hits, rgba, _, pos, vox = oracle_mod.render_ex(osvo, ocam, w, h, mode)
    return hits, rgba, pos, vox


def _bufs(torch, n_px):
    """Every output buffer, pre-filled with a pattern no render produces.  The fills
    run on torch's stream and the plugin renders on its context's own non-blocking
    stream, which does not wait for torch's: synchronize before handing them over."""
    t = torch
    b = {"hits": t.full((n_px * 24,), 0xA5, dtype=t.uint8, device="cuda"),
         "rgba": t.full((n_px * 4,), -7.0, dtype=t.float32, device="cuda"),
         "rgba8": t.full((n_px,), 0x1234567, dtype=t.int32, device="cuda"),
         "compact": t.full((n_px * 12,), 0x5A, dtype=t.uint8, device="cuda"),
         "position": t.full((n_px * 4,), -9.0, dtype=t.float32, device="cuda"),
         "voxel": t.full((n_px,), 77, dtype=t.int64, device="cuda"),
         "rgb8": t.full((n_px * 3,), 0xA5, dtype=t.uint8, device="cuda")}
    t.cuda.synchronize()
    return b


def _ptrs(b, keys=None):
    return {k: v.data_ptr() for k, v in b.items() if keys is None or k in keys}


def _check(b, oracle_mod, ref_hits, ref_rgba, ref_pos=None, ref_vox=None, keys=None):
    keys = set(b) if keys is None else set(keys)
    hits = b["hits"].cpu().numpy().view(HIT_DTYPE)
    if "hits" in keys:
        bad = np.flatnonzero(hits.view(np.uint8).reshape(-1, 24).any(axis=1) &
                             (hits.tobytes() != ref_hits.tobytes()))
        assert hits.tobytes() == ref_hits.tobytes(), f"hit records differ ({len(bad)} px)"
    if "rgba" in keys:
        assert b["rgba"].cpu().numpy().tobytes() == ref_rgba.astype(np.float32).tobytes(), "Result differs"
    if "rgba8" in keys:
        got = b["rgba8"].cpu().numpy().view(np.uint32)
        assert np.array_equal(got, oracle_mod.pack_rgba8(ref_rgba)), "RGBA8 differs"
    if "compact" in keys:
        c = b["compact"].cpu().numpy().reshape(-1, 12)
        assert c.tobytes() == ref_hits.view(np.uint8).reshape(-1, 24)[:, :12].tobytes(), "compact differs"
    if "position" in keys and ref_pos is not None:
        assert b["position"].cpu().numpy().tobytes() == ref_pos.tobytes(), "position differs"
    if "rgb8" in keys:
        got = b["rgb8"].cpu().numpy().reshape(-1, 3)
        want = oracle_mod.pack_rgba8(ref_rgba).view(np.uint8).reshape(-1, 4)[:, :3]
        assert np.array_equal(got, want), "RGB8 differs"
    if "voxel" in keys and ref_vox is not None:
        assert np.array_equal(b["voxel"].cpu().numpy().view(np.uint64), ref_vox), "voxel key differs"


def test_each_output_alone_matches_oracle(torch, oracle_mod):
    """Every output requested on its own (nothing computed only for another
    output): the display words and the RGB payload carry the shaded colour even
    without the Result, the compact record without the hit record."""
    svo = build_menger(8)
    w, h = 333, 201
    cam = overview_camera()
    ref_hits, ref_rgba, ref_pos, ref_vox = _oracle(oracle_mod, svo, cam, w, h)
    m = RaytracingMaster(device=0, capacity_nodes=len(svo))
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        for key in ("hits", "rgba", "rgba8", "rgb8", "compact", "position", "voxel"):
            b = _bufs(torch, w * h)
            m.render_frame(w, h, **_ptrs(b, (key,)))
            m.synchronize()
            _check(b, oracle_mod, ref_hits, ref_rgba, ref_pos, ref_vox, keys=(key,))
    finally:
        m.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_every_output_matches_oracle(torch, oracle_mod, text_svo, mode):
    """All seven outputs of one launch, Text SVO (C1) and the 256^3 Menger (V2)."""
    for svo, cam, (w, h) in ((text_svo, main_camera(), (256, 256)), (text_svo, overview_camera(), (300, 200)),
                             (build_menger(8), overview_camera(), (480, 272))):
        ref_hits, ref_rgba, ref_pos, ref_vox = _oracle(oracle_mod, svo, cam, w, h, mode)
        assert np.count_nonzero(ref_hits["flags"] & 1) > 500
        m = RaytracingMaster(device=0, capacity_nodes=len(svo))
        try:
            m.SetSVOBuffer(svo)
            m.UpdateShaderParameters(cam, w, h)
            b = _bufs(torch, w * h)
            for _ in range(3):   # cost-ordered relaunches too
                m.render_frame(w, h, stack_mode=mode, **_ptrs(b))
                m.synchronize()
                _check(b, oracle_mod, ref_hits, ref_rgba, ref_pos, ref_vox)
        finally:
            m.close()


def test_voxel_key_and_position_properties(torch, oracle_mod):
    """Size-independent properties of the new outputs on the 256^3 Menger: the
    key's voxel box contains the hit position, its scale is the leaf scale,
    misses carry position 0 and key ~0."""
    svo = build_menger(8)
    cam = overview_camera()
    w, h = 640, 360
    m = RaytracingMaster(device=0, capacity_nodes=len(svo))
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        b = _bufs(torch, w * h)
        m.render_frame(w, h, **_ptrs(b, ("hits", "position", "voxel")))
        m.synchronize()
    finally:
        m.close()
    hits = b["hits"].cpu().numpy().view(HIT_DTYPE)
    pos = b["position"].cpu().numpy().reshape(-1, 4)
    vox = b["voxel"].cpu().numpy().view(np.uint64)
    hit = (hits["flags"] & 1) != 0
    assert hit.sum() > 1000 and (~hit).sum() > 1000
    assert np.all(vox[~hit] == np.uint64(0xFFFFFFFFFFFFFFFF)) and np.all(pos[~hit] == 0)
    depth = 23 - hits["hit_scale"][hit].astype(np.int64)
    assert np.all(depth == 8)
    k = np.stack([(vox[hit] >> np.uint64(21 * a)) & np.uint64((1 << 21) - 1) for a in range(3)], 1).astype(np.float64)
    c = pos[hit, :3].astype(np.float64) / 64.0 + 1.5
    lo = 1.0 + k / 256.0
    assert np.all((c >= lo - 1e-6) & (c <= lo + 1.0 / 256.0 + 1e-6))


def test_frame_layout_bands_fill_the_frame(torch, text_svo):
    """Band renders written in place into full-frame buffers (SVO_LAYOUT_FRAME)
    give exactly the whole-frame render, and leave other rows untouched."""
    cam = overview_camera()
    w, h = 200, 150
    m = RaytracingMaster(device=0, capacity_nodes=len(text_svo))
    try:
        m.SetSVOBuffer(text_svo)
        m.UpdateShaderParameters(cam, w, h)
        full_rgba, full = m.Render(w, h)
        b = _bufs(torch, w * h)
        m.render_frame(w, h, hits=b["hits"].data_ptr(), rgba8=b["rgba8"].data_ptr(), layout=_lib.LAYOUT_FRAME,
                       band=(8, 1, 3))
        m.synchronize()
        got = b["hits"].cpu().numpy().view(HIT_DTYPE).reshape(h, w)
        ys = band_rows(h, (8, 1, 3))
        other = np.setdiff1d(np.arange(h), ys)
        assert got[ys].tobytes() == full[ys].tobytes()
        assert np.all(got[other].view(np.uint8) == 0xA5)
        for r in (0, 2):
            m.render_frame(w, h, hits=b["hits"].data_ptr(), layout=_lib.LAYOUT_FRAME, band=(8, r, 3))
        m.synchronize()
        assert b["hits"].cpu().numpy().tobytes() == full.tobytes()
    finally:
        m.close()


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0, 0, 0]])
def test_multi_device_context_matches_oracle(torch, oracle_mod, text_svo, devices):
    """svo_create_multi with the device repeated: the bands of members 1.. are
    rendered into double-buffered payloads and pulled by the display member's
    assemble kernel (compact records when hit records / Result are asked for,
    RGBA8 words for a display-only frame).  Frames alternate cameras so a stale
    payload would show."""
    svo = build_menger(8)
    w, h = 333, 250
    cams = [overview_camera(), Camera(position=(30.0, 12.0, -25.0), rotation=look_rotation((-30.0, -12.0, 25.0)))]
    refs = [_oracle(oracle_mod, svo, c, w, h) for c in cams]
    m = RaytracingMaster(devices=devices, capacity_nodes=len(svo))
    try:
        assert m.num_devices() == len(devices)
        m.SetSVOBuffer(svo)
        for i in range(6):
            cam = cams[i % 2]
            ref_hits, ref_rgba, _, _ = refs[i % 2]
            m.UpdateShaderParameters(cam, w, h)
            rgba, hits = m.Render(w, h)                       # host path: svo_render
            assert hits.tobytes() == ref_hits.tobytes()
            assert rgba.reshape(-1, 4).tobytes() == ref_rgba.tobytes()
            b = _bufs(torch, w * h)
            m.render_frame(w, h, rgba8=b["rgba8"].data_ptr(), layout=_lib.LAYOUT_FRAME)    # display-only payload
            m.render_frame(w, h, compact=b["compact"].data_ptr(), hits=b["hits"].data_ptr(),
                           layout=_lib.LAYOUT_FRAME)
            m.synchronize()
            _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba8", "compact"))
        for k in range(len(devices)):
            assert m.member(k).info()["n_nodes"] == len(svo)
    finally:
        m.close()


def test_multi_device_payload_regrowth_across_streams(torch, oracle_mod):
    """Frames of growing size on alternating caller streams: a larger frame
    reallocates the members' payloads, which the display member's assembles of
    the earlier frames -- queued on the OTHER caller stream -- may still read;
    the plugin waits for those assembles (their events), not for this call's
    stream.  Every frame equals the oracle's."""
    svo = build_menger(8)
    cam = overview_camera()
    sizes = [(96, 64), (200, 120), (333, 250), (96, 64), (480, 272)]
    refs = {wh: _oracle(oracle_mod, svo, cam, *wh) for wh in set(sizes)}
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    m = RaytracingMaster(devices=[0, 0, 0], capacity_nodes=len(svo))
    try:
        m.SetSVOBuffer(svo)
        frames = []
        for i, (w, h) in enumerate(sizes):
            m.UpdateShaderParameters(cam, w, h)
            f = torch.full((w * h,), 0x1234567, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()   # the fill before the plugin's stream writes the frame
            m.render_frame(w, h, rgba8=f.data_ptr(), layout=_lib.LAYOUT_FRAME, stream=streams[i % 2].cuda_stream)
            frames.append(f)
        m.synchronize()
        torch.cuda.synchronize()
        for (w, h), f in zip(sizes, frames):
            got = f.cpu().numpy().view(np.uint32)
            assert np.array_equal(got, oracle_mod.pack_rgba8(refs[(w, h)][1])), f"{w}x{h} RGBA8 differs"
    finally:
        m.close()


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0, 0, 0]])
def test_multi_device_sparse_payload(torch, oracle_mod, devices):
    """svo_config.sparse_payload 1: the multi-device context's display-only frames travel as
    sparse parts (masks + offsets + hit RGB, packed on each member) that the display
    member's assemble pulls with no host round trip -- round-robin and weighted
    deals, frames alternating cameras (a stale part would show), bit-identical to
    the oracle."""
    from raytracingtest_amd.distributed import weighted_owner
    svo = build_menger(8)
    w, h = 333, 250
    cams = [overview_camera(), Camera(position=(30.0, 12.0, -25.0), rotation=look_rotation((-30.0, -12.0, 25.0)))]
    refs = [_oracle(oracle_mod, svo, c, w, h) for c in cams]
    m = RaytracingMaster(devices=devices, capacity_nodes=len(svo), config={"sparse_payload": 1})
    try:
        m.SetSVOBuffer(svo)
        for owner in (None, weighted_owner(len(devices), 3 / 8)):
            m.set_band_deal(owner)
            for i in range(4):
                ref_hits, ref_rgba, _, _ = refs[i % 2]
                m.UpdateShaderParameters(cams[i % 2], w, h)
                b = _bufs(torch, w * h)
                m.render_frame(w, h, rgba8=b["rgba8"].data_ptr(), layout=_lib.LAYOUT_FRAME)
                m.synchronize()
                _check(b, oracle_mod, ref_hits, ref_rgba, keys=("rgba8",))
        # with the '+1 shadow ray' pass: occluded hits travel as black RGB in the sparse parts
        sh_hits, sh_rgba, _, _ = _oracle(oracle_mod, svo, cams[0], w, h, shadows=True)
        m.UpdateShaderParameters(cams[0], w, h)
        m.SetShadowRays(True)
        b = _bufs(torch, w * h)
        m.render_frame(w, h, rgba8=b["rgba8"].data_ptr(), layout=_lib.LAYOUT_FRAME)
        m.synchronize()
        _check(b, oracle_mod, sh_hits, sh_rgba, keys=("rgba8",))
    finally:
        m.close()


def test_multi_device_weighted_deal(torch, oracle_mod):
    """svo_set_band_deal: a three-member context whose display member takes 3 of
    every 8 rounds' bands (it also assembles) renders the same frame as the
    oracle, for the compact (hit records + Result) and RGBA8 payloads, and a
    bad owner table is refused."""
    from raytracingtest_amd.distributed import weighted_owner
    svo = build_menger(8)
    w, h = 300, 250
    cam = overview_camera()
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h)
    m = RaytracingMaster(devices=[0, 0, 0], capacity_nodes=len(svo))
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        for owner in (weighted_owner(3, 3 / 8), None, weighted_owner(3, 1 / 8)):
            m.set_band_deal(owner)
            rgba, hits = m.Render(w, h)
            assert hits.tobytes() == ref_hits.tobytes()
            assert rgba.reshape(-1, 4).tobytes() == ref_rgba.tobytes()
            b = _bufs(torch, w * h)
            m.render_frame(w, h, rgba8=b["rgba8"].data_ptr(), layout=_lib.LAYOUT_FRAME)
            m.synchronize()
            _check(b, oracle_mod, ref_hits, ref_rgba, keys=("rgba8",))
        with pytest.raises(SvoError):
            m.set_band_deal([0, 1, 3])
    finally:
        m.close()


@pytest.mark.parametrize("compact", [False, True])
def test_multi_device_shadow_rays(torch, oracle_mod, compact):
    """The C3 '+1 shadow ray' frame through the multi-device context: the
    occlusion flag travels in the compact record and the display member
    rebuilds the black Result."""
    svo = build_menger(8)
    w, h = 400, 240
    cam = overview_camera()
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h, shadows=True)
    # compact: every member's shadow pass over its bands' compacted hit list
    m = RaytracingMaster(devices=[0, 0, 0], capacity_nodes=len(svo), config={"shadow_form": 2 if compact else 0})
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        m.SetShadowRays(True)
        rgba, hits = m.Render(w, h)
        assert np.count_nonzero(hits.reshape(-1)["flags"] & 8) > 0
        assert hits.tobytes() == ref_hits.tobytes()
        assert rgba.reshape(-1, 4).tobytes() == ref_rgba.tobytes()
    finally:
        m.close()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_assemble_from_rank_parts(torch, oracle_mod, world):
    """The one-process-per-GPU split: each 'rank' renders its bands (band
    layout) into a compact and an RGBA8 payload; svo_assemble_frame rebuilds the
    frame from the parts -- what bench.py's rank 0 does after the RCCL gather."""
    svo = build_menger(7)
    cam = overview_camera()
    w, h = 256, 200
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h)
    m = RaytracingMaster(device=0, capacity_nodes=len(svo))
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        comp, rgb8, rgb3 = [], [], []
        for r in range(world):
            n = len(band_rows(h, (8, r, world))) * w
            comp.append(torch.zeros(max(n, 1) * 12, dtype=torch.uint8, device="cuda"))
            rgb8.append(torch.zeros(max(n, 1), dtype=torch.int32, device="cuda"))
            rgb3.append(torch.zeros(max(n, 1) * 3, dtype=torch.uint8, device="cuda"))
            torch.cuda.synchronize()   # the zero fills (torch's stream) before the plugin's stream writes
            m.render_frame(w, h, compact=comp[-1].data_ptr(), rgba8=rgb8[-1].data_ptr(), rgb8=rgb3[-1].data_ptr(),
                           band=(8, r, world))
        b = _bufs(torch, w * h)
        m.assemble_frame(w, h, [c.data_ptr() for c in comp], _lib.PART_COMPACT, hits=b["hits"].data_ptr(),
                         rgba=b["rgba"].data_ptr(), compact=b["compact"].data_ptr())
        b2 = _bufs(torch, w * h)
        m.assemble_frame(w, h, [c.data_ptr() for c in rgb8], _lib.PART_RGBA8, rgba8=b2["rgba8"].data_ptr())
        # bench.py's display rank: its own bands rendered straight into the frame, the
        # other parts assembled around them (skip_part 0)
        b3 = _bufs(torch, w * h)
        m.render_frame(w, h, rgba8=b3["rgba8"].data_ptr(), layout=_lib.LAYOUT_FRAME, band=(8, 0, world))
        m.assemble_frame(w, h, [None] + [c.data_ptr() for c in rgb8[1:]], _lib.PART_RGBA8,
                         rgba8=b3["rgba8"].data_ptr(), skip_part=0)
        b4 = _bufs(torch, w * h)   # 3-byte RGB parts (the default N > 1 payload)
        m.assemble_frame(w, h, [c.data_ptr() for c in rgb3], _lib.PART_RGB8, rgba8=b4["rgba8"].data_ptr())
        m.synchronize()
        _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba", "compact"))
        _check(b2, oracle_mod, ref_hits, ref_rgba, keys=("rgba8",))
        _check(b3, oracle_mod, ref_hits, ref_rgba, keys=("rgba8",))
        _check(b4, oracle_mod, ref_hits, ref_rgba, keys=("rgba8",))
        with pytest.raises(_lib.SvoError):   # RGBA8 parts cannot rebuild hit records
            m.assemble_frame(w, h, [c.data_ptr() for c in rgb8], _lib.PART_RGBA8, hits=b["hits"].data_ptr())
    finally:
        m.close()


@pytest.mark.parametrize("world,share", [(2, 0.625), (3, 0.5), (8, 0.75)])
def test_weighted_deal_parts_match_oracle(torch, oracle_mod, world, share):
    """bench.py's weighted deal (the display rank renders fewer bands): parts
    rendered with the owner table in svo_band, the display rank's own rows
    straight into the frame, the rest assembled by svo_assemble_frame with the
    same table -- RGBA8 and compact parts, both bit-identical to one frame."""
    from raytracingtest_amd.distributed import weighted_owner
    svo = build_menger(7)
    cam = overview_camera()
    w, h = (262 if world == 3 else 264), 203   # 262: rows not 16-byte multiples (per-pixel assemble path)
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h)
    owner = weighted_owner(world, share)
    m = RaytracingMaster(device=0, capacity_nodes=len(svo))
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        b = _bufs(torch, w * h)
        m.render_frame(w, h, hits=b["hits"].data_ptr(), rgba=b["rgba"].data_ptr(), rgba8=b["rgba8"].data_ptr(),
                       layout=_lib.LAYOUT_FRAME, band=(8, 0, world, owner))
        comp, rgb8, rgb3 = [None], [None], [None]
        for r in range(1, world):
            n = len(band_rows(h, (8, r, world, owner))) * w
            comp.append(torch.zeros(max(n, 1) * 12, dtype=torch.uint8, device="cuda"))
            rgb8.append(torch.zeros(max(n, 1), dtype=torch.int32, device="cuda"))
            rgb3.append(torch.zeros(max(n, 1) * 3, dtype=torch.uint8, device="cuda"))
            torch.cuda.synchronize()   # the zero fills (torch's stream) before the plugin's stream writes
            m.render_frame(w, h, compact=comp[-1].data_ptr(), rgba8=rgb8[-1].data_ptr(), rgb8=rgb3[-1].data_ptr(),
                           band=(8, r, world, owner))
        b2 = _bufs(torch, w * h)
        m.render_frame(w, h, rgba8=b2["rgba8"].data_ptr(), layout=_lib.LAYOUT_FRAME, band=(8, 0, world, owner))
        m.assemble_frame(w, h, [None] + [c.data_ptr() for c in rgb8[1:]], _lib.PART_RGBA8,
                         rgba8=b2["rgba8"].data_ptr(), skip_part=0, owner=owner)
        m.assemble_frame(w, h, [None] + [c.data_ptr() for c in comp[1:]], _lib.PART_COMPACT,
                         hits=b["hits"].data_ptr(), rgba=b["rgba"].data_ptr(), rgba8=b["rgba8"].data_ptr(),
                         skip_part=0, owner=owner)
        b3 = _bufs(torch, w * h)
        m.render_frame(w, h, rgba8=b3["rgba8"].data_ptr(), layout=_lib.LAYOUT_FRAME, band=(8, 0, world, owner))
        m.assemble_frame(w, h, [None] + [c.data_ptr() for c in rgb3[1:]], _lib.PART_RGB8,
                         rgba8=b3["rgba8"].data_ptr(), skip_part=0, owner=owner)
        m.synchronize()
        _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba", "rgba8"))
        _check(b2, oracle_mod, ref_hits, ref_rgba, keys=("rgba8",))
        _check(b3, oracle_mod, ref_hits, ref_rgba, keys=("rgba8",))
        with pytest.raises(SvoError):   # owner entry naming a rank outside the deal
            m.render_frame(w, h, rgba8=b2["rgba8"].data_ptr(), band=(8, 0, world, [0, world]))
    finally:
        m.close()


def _sparse_part(torch, m, w, h, band):
    """A rank's sparse payload: render the dense RGB + the tile hit masks (at the
    part's head), then svo_pack_hits.  Returns (part, offsets incl. the count, n_tiles)."""
    rows = len(band_rows(h, band))
    n_tiles = ((w + 7) // 8) * ((rows + 7) // 8)
    dense = torch.full((max(rows * w, 1) * 3,), 0xA5, dtype=torch.uint8, device="cuda")
    part = torch.full((_lib.sparse_part_bytes(n_tiles, rows * w),), 0x5A, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()   # the fills before the plugin's stream writes
    m.render_frame(w, h, rgb8=dense.data_ptr(), hitmask=part.data_ptr(), band=band)
    m.pack_hits(w, h, band, dense.data_ptr(), part.data_ptr())
    return part, part[8 * n_tiles:12 * n_tiles + 4].view(torch.int32), n_tiles


@pytest.mark.parametrize("world,share", [(1, None), (2, None), (3, 0.5), (8, 0.75)])
def test_sparse_parts_match_oracle(torch, oracle_mod, world, share):
    """The sparse band payload (tile hit masks + the RGB of hit pixels only):
    each rank's hit count equals the oracle's hits in its rows, the packed
    colours are the hits' RGBA8 bytes in tile/lane order, and the display rank
    rebuilds the frame (misses: sky computed there) bit-identical to one frame
    -- round-robin and weighted deals, frame widths that are not tile multiples."""
    from raytracingtest_amd.distributed import weighted_owner
    svo = build_menger(7)
    cam = overview_camera()
    w, h = {1: (1000, 600), 3: (262, 203)}.get(world, (264, 200))   # 1000x600: 9,375 tiles, a 10-chunk scan
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h)
    ref_hit = ((ref_hits["flags"] & 1) != 0).reshape(h, w)
    ref_rgb = oracle_mod.pack_rgba8(ref_rgba).view(np.uint8).reshape(h, w, 4)[:, :, :3]
    owner = None if share is None else weighted_owner(world, share)
    m = RaytracingMaster(device=0, capacity_nodes=len(svo))
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        parts = []
        for r in range(world):
            band = (8, r, world) if owner is None else (8, r, world, owner)
            part, offs, n_tiles = _sparse_part(torch, m, w, h, band)
            parts.append(part)
            m.synchronize()
            ys = band_rows(h, band)
            count = int(offs[n_tiles].item())
            assert count == int(ref_hit[ys].sum())
            # the packed colours: tiles in order, lanes (row-major 8x8) within a tile
            tx = (w + 7) // 8
            want = []
            for t in range(n_tiles):
                by, bx = divmod(t, tx)
                for lane in range(64):
                    ly, lx = by * 8 + lane // 8, bx * 8 + lane % 8
                    if ly < len(ys) and lx < w and ref_hit[ys[ly], lx]:
                        want.append(ref_rgb[ys[ly], lx])
            head = _lib.sparse_head_bytes(n_tiles)
            got = part[head:head + 3 * count].cpu().numpy().reshape(-1, 3)
            assert np.array_equal(got, np.array(want, np.uint8).reshape(-1, 3))
        b = _bufs(torch, w * h)
        m.assemble_frame(w, h, [p.data_ptr() for p in parts], _lib.PART_SPARSE_RGB8, rgba8=b["rgba8"].data_ptr(),
                         owner=owner)
        b2 = _bufs(torch, w * h)   # the display rank's own rows rendered in place
        band0 = (8, 0, world) if owner is None else (8, 0, world, owner)
        m.render_frame(w, h, rgba8=b2["rgba8"].data_ptr(), layout=_lib.LAYOUT_FRAME, band=band0)
        m.assemble_frame(w, h, [None] + [p.data_ptr() for p in parts[1:]], _lib.PART_SPARSE_RGB8,
                         rgba8=b2["rgba8"].data_ptr(), skip_part=0, owner=owner)
        m.synchronize()
        _check(b, oracle_mod, ref_hits, ref_rgba, keys=("rgba8",))
        _check(b2, oracle_mod, ref_hits, ref_rgba, keys=("rgba8",))
        with pytest.raises(SvoError):   # sparse parts rebuild only display words
            m.assemble_frame(w, h, [p.data_ptr() for p in parts], _lib.PART_SPARSE_RGB8, hits=b["hits"].data_ptr())
    finally:
        m.close()


@pytest.mark.parametrize("mode", [0, 1])
def test_sparse_parts_with_shadow_rays(torch, oracle_mod, mode):
    """The sparse payload of the C3 '+1 shadow ray' frame: occluded hits travel
    as black RGB, both stack modes, and the frame rebuilds bit-identically."""
    svo = build_menger(8)
    cam = overview_camera()
    w, h = 400, 240
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h, mode, shadows=True)
    assert np.count_nonzero(ref_hits["flags"] & 8) > 0
    m = RaytracingMaster(device=0, capacity_nodes=len(svo))
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        m.SetShadowRays(True)
        parts = []
        for r in range(3):
            band = (8, r, 3)
            rows = len(band_rows(h, band))
            n_tiles = ((w + 7) // 8) * ((rows + 7) // 8)
            dense = torch.empty(rows * w * 3, dtype=torch.uint8, device="cuda")
            part = torch.empty(_lib.sparse_part_bytes(n_tiles, rows * w), dtype=torch.uint8, device="cuda")
            m.render_frame(w, h, rgb8=dense.data_ptr(), hitmask=part.data_ptr(), band=band, stack_mode=mode)
            m.pack_hits(w, h, band, dense.data_ptr(), part.data_ptr())
            parts.append(part)
        b = _bufs(torch, w * h)
        m.assemble_frame(w, h, [p.data_ptr() for p in parts], _lib.PART_SPARSE_RGB8, rgba8=b["rgba8"].data_ptr())
        m.synchronize()
        _check(b, oracle_mod, ref_hits, ref_rgba, keys=("rgba8",))
    finally:
        m.close()


@pytest.mark.parametrize("w,rows", [(7680, 1080), (64, 8), (13, 3), (1000, 7)])
def test_pack_hits_random_masks(torch, w, rows):
    """svo_pack_hits on random masks and colours (no render): the offsets are the
    exclusive prefix sum of the tiles' popcounts over a multi-chunk scan (7680 x
    1080: 129,600 tiles), the count is the total, and the packed bytes are the hit
    pixels' RGB in tile / lane order; pixels outside the band's width or rows
    never count."""
    rng = np.random.default_rng(w * 31 + rows)
    tx, ty = (w + 7) // 8, (rows + 7) // 8
    n_tiles = tx * ty
    lane_ok = np.zeros((ty, tx, 64), bool)
    for lane in range(64):
        ly, lx = np.arange(ty)[:, None] * 8 + lane // 8, np.arange(tx)[None, :] * 8 + lane % 8
        lane_ok[:, :, lane] = (ly < rows) & (lx < w)
    density = rng.uniform(0.0, 1.0, (ty, tx, 1))
    bits = (rng.uniform(0.0, 1.0, (ty, tx, 64)) < density) & lane_ok
    masks = (bits.astype(np.uint64) << np.arange(64, dtype=np.uint64)).sum(axis=2, dtype=np.uint64).reshape(-1)
    rgb = rng.integers(0, 256, (rows, w, 3), dtype=np.uint8)
    m = RaytracingMaster(device=0, capacity_nodes=16)
    try:
        part = torch.full((_lib.sparse_part_bytes(n_tiles, rows * w),), 0xEE, dtype=torch.uint8, device="cuda")
        part[:n_tiles * 8] = torch.from_numpy(masks.view(np.uint8)).cuda()
        dense = torch.from_numpy(rgb.reshape(-1)).cuda()
        torch.cuda.synchronize()   # torch's copies before the plugin's stream reads them
        m.pack_hits(w, rows, (8, 0, 1), dense.data_ptr(), part.data_ptr())
        m.synchronize()
        offs = part[8 * n_tiles:12 * n_tiles + 4].view(torch.int32)
        cnt = bits.reshape(n_tiles, 64).sum(axis=1)
        want_off = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
        got_off = offs[:n_tiles + 1].cpu().numpy().astype(np.int64)
        assert np.array_equal(got_off, want_off)
        t, lane = np.nonzero(bits.reshape(n_tiles, 64))
        ys = (t // tx) * 8 + lane // 8
        xs = (t % tx) * 8 + lane % 8
        head = _lib.sparse_head_bytes(n_tiles)
        got = part[head:head + 3 * int(want_off[-1])].cpu().numpy().reshape(-1, 3)
        assert np.array_equal(got, rgb[ys, xs])
    finally:
        m.close()


@pytest.mark.parametrize("pose", ["all_miss", "all_hit"])
def test_sparse_parts_extremes(torch, oracle_mod, pose):
    """Sparse payload edge cases: a frame with no hit (the part is the masks
    alone, count 0) and a frame hit everywhere (the part is as large as the
    dense RGB plus the masks); both rebuild the oracle's frame."""
    from raytracingtest_amd.builder import build_menger as menger
    svo = menger(6, levels=0)   # a solid cube
    if pose == "all_miss":
        cam = overview_camera(target=(0.0, 60.0, -80.0))
    else:
        cam = overview_camera()
        cam.fov = 5.0
    w, h = 200, 120
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h)
    n_hit = int(np.count_nonzero(ref_hits["flags"] & 1))
    assert n_hit == (0 if pose == "all_miss" else w * h)
    m = RaytracingMaster(device=0, capacity_nodes=len(svo))
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        parts = []
        for r in range(2):
            part, offs, nt = _sparse_part(torch, m, w, h, (8, r, 2))
            parts.append(part)
            m.synchronize()
            assert int(offs[nt].item()) == (0 if pose == "all_miss" else len(band_rows(h, (8, r, 2))) * w)
        b = _bufs(torch, w * h)
        m.assemble_frame(w, h, [p.data_ptr() for p in parts], _lib.PART_SPARSE_RGB8, rgba8=b["rgba8"].data_ptr())
        m.synchronize()
        _check(b, oracle_mod, ref_hits, ref_rgba, keys=("rgba8",))
    finally:
        m.close()


@pytest.mark.parametrize("n_streams", [2, 6])
def test_two_streams_every_pixel_written(torch, oracle_mod, n_streams):
    """Launches of one context cycling over several streams (advisor r1): each
    stream has its own dispatch-order state (up to 4; a fifth stream takes over
    the least recently used set after that stream's renders), the orders are
    rebuilt every launch (order_every 1), the renders run concurrently, and
    every frame is still complete and equal to the oracle's."""
    svo = build_menger(8)
    m = RaytracingMaster(device=0, capacity_nodes=len(svo), config={"order_every": 1})
    w, h = 640, 360
    cam = overview_camera()
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h)
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        streams = [torch.cuda.Stream() for _ in range(n_streams)]
        outs = [_bufs(torch, w * h) for _ in range(3 * n_streams)]
        for i, b in enumerate(outs):
            m.render_frame(w, h, hits=b["hits"].data_ptr(), rgba=b["rgba"].data_ptr(),
                           stream=streams[i % n_streams].cuda_stream)
        torch.cuda.synchronize()
        for b in outs:
            _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba"))
    finally:
        m.close()


def test_forgotten_streams_destroyed_then_new_ones(torch, oracle_mod):
    """a caller stream must stay alive until svo_forget_stream.  Four streams fill the
    context's dispatch-order sets, each is forgotten and destroyed, then six fresh streams (HIP
    may reuse the old handles) render again: no event lands on a dead stream, every frame is
    complete and equal to the oracle's, and forgetting an unknown stream is not an error."""
    svo = build_menger(8)
    w, h = 320, 184
    cam = overview_camera()
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h)
    m = RaytracingMaster(device=0, capacity_nodes=len(svo))
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        for generation in range(2):
            streams = [torch.cuda.Stream() for _ in range(4 if generation == 0 else 6)]
            outs = [_bufs(torch, w * h) for _ in range(2 * len(streams))]
            for i, b in enumerate(outs):
                m.render_frame(w, h, hits=b["hits"].data_ptr(), rgba=b["rgba"].data_ptr(),
                               stream=streams[i % len(streams)].cuda_stream)
            for st in streams:
                m.forget_stream(st.cuda_stream)
            for b in outs:   # forget_stream waited for each stream's renders
                _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba"))
            del streams
        m.forget_stream(torch.cuda.Stream().cuda_stream)
    finally:
        m.close()


def _hip_runtime():
    """The HIP runtime this process already loaded (torch's or /opt/rocm's: one soname), for raw
    stream handles that a test can really destroy (torch pools its streams and never does)."""
    import ctypes
    path = None
    with open("/proc/self/maps") as fh:
        for line in fh:
            if "libamdhip64" in line:
                path = line.split()[-1]
                break
    assert path, "no HIP runtime loaded"
    hip = ctypes.CDLL(path)
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    return hip


@pytest.mark.parametrize("release", ["synchronize", "forget"])
def test_raw_streams_destroyed_after_forget_or_synchronize(torch, oracle_mod, release):
    """a host that follows the stream-lifetime rule (svo_rt.h) -- svo_synchronize, or
    svo_forget_stream per stream, then hipStreamDestroy -- and renders on fresh streams until the
    dispatch-order sets are evicted (six streams after four) and the host-path scratch moves (the
    two-pass shadow form without caller hit records uses it, then svo_render on the context's own
    stream): no event may land on a destroyed handle (HIP may hand the same value to a new stream),
    and every frame equals the oracle's.  Raw hipStreamCreate handles, really destroyed."""
    import ctypes
    hip = _hip_runtime()
    svo = build_menger(8)
    w, h = 320, 184
    cam = overview_camera()
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h)
    sh_hits, sh_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h, shadows=True)
    m = RaytracingMaster(device=0, capacity_nodes=len(svo), config={"shadow_form": 1})
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        for generation in range(3):
            streams = []
            for _ in range(4 if generation == 0 else 6):
                hs = ctypes.c_void_p()
                assert hip.hipStreamCreate(ctypes.byref(hs)) == 0
                streams.append(hs.value)
            outs = [_bufs(torch, w * h) for _ in range(2 * len(streams))]
            for i, b in enumerate(outs):
                m.render_frame(w, h, hits=b["hits"].data_ptr(), rgba=b["rgba"].data_ptr(),
                               stream=streams[i % len(streams)])
            # the scratch: shadow rays as a second pass need records the caller did not ask for
            m.SetShadowRays(True)
            sh = _bufs(torch, w * h)
            m.render_frame(w, h, rgba=sh["rgba"].data_ptr(), stream=streams[0])
            m.SetShadowRays(False)
            if release == "synchronize":
                m.synchronize()
            else:
                for st in streams:
                    m.forget_stream(st)
            for st in streams:
                assert hip.hipStreamDestroy(st) == 0
            for b in outs:
                _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba"))
            assert sh["rgba"].cpu().numpy().tobytes() == sh_rgba.astype(np.float32).tobytes()
            rgba, hits = m.Render(w, h)   # the context's own stream takes the scratch over
            assert hits.tobytes() == ref_hits.tobytes()
    finally:
        m.close()


def test_config_change_takes_effect(torch, oracle_mod, monkeypatch, capfd):
    """policy set through the ABI (svo_set_config) on a live context, with no
    policy environment variable, changes what the next launches do -- beam starts off / on (the
    starts svo_beam_starts reports and the fetches the beam-started walk makes), the segment class
    table each launch dispatches in (the SVO_DEBUG order trace, a diagnostic), the readback form --
    while every frame stays the oracle's; out-of-range fields are refused and change nothing."""
    import re
    from raytracingtest_amd import _lib
    from raytracingtest_amd.native_builder import build_sampler_svo
    monkeypatch.setenv("SVO_DEBUG", "2")   # diagnostics only: the order trace
    svo = build_sampler_svo(4, 11)   # C3's pool and frame: heavy chains, so every class table applies
    w, h = 1920, 1080
    cam = CAMERAS["flyover"]()
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h)
    m = RaytracingMaster(device=0, capacity_nodes=len(svo))
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        assert m.get_config() == _lib.default_config()
        starts = torch.empty(w * h, dtype=torch.float32, device="cuda")
        fetch = torch.zeros(w * h, dtype=torch.int32, device="cuda")

        def probe():
            m.beam_starts_device(w, h, starts.data_ptr())
            m.set_count_beam(True)
            m.count_fetches_device(w, h, fetch.data_ptr())
            m.set_count_beam(False)
            m.synchronize()
            return int(np.isfinite(starts.cpu().numpy()).sum()), int(fetch.to(torch.int64).sum().item())

        def frames(n=4):
            capfd.readouterr()
            for _ in range(n):
                b = _bufs(torch, w * h)
                m.render_frame(w, h, hits=b["hits"].data_ptr(), rgba=b["rgba"].data_ptr())
                m.synchronize()
                _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba"))
            return [int(k, 16) for k in re.findall(r"svo order: .* kpack ([0-9a-f]+) ", capfd.readouterr().err)]

        beam_rays, beam_fetches = probe()
        assert beam_rays > 0
        frames()
        m.set_config(beam=0)
        off_rays, off_fetches = probe()
        assert off_rays == 0 and off_fetches > beam_fetches   # every ray from the cube entry
        frames()
        m.set_config(beam=1, beam_back=1)                     # rebuilt from the device copy
        back_rays, back_fetches = probe()
        assert 0 < back_rays <= beam_rays and back_fetches < off_fetches
        m.set_config(seg_table_issue=0x888, seg_table_latency=0x888, seg_table_thin=0x888)
        assert frames(6)[-1] == 0x888
        m.set_config(segments=0)
        assert frames(3)[-1] == 0
        before = m.get_config()
        for bad in ({"seg_table_issue": 0x5}, {"order_every": 0}, {"shadow_form": 3}, {"lat_ratio": float("nan")}):
            with pytest.raises(SvoError):
                m.set_config(**bad)
            assert m.get_config() == before
        m.set_config(readback=2)
        m.RenderProgressiveAsync(w, h)
        m.RenderProgressiveAsync(w, h)
        got = m.ProgressiveLast(w, h)
        assert got is not None and got.shape == (h, w)
    finally:
        m.close()


def _rand_subtree(rng, depth, nodes, att, p_leaf=0.5):
    """Append a random V2 subtree of exactly `depth` descriptor levels (one
    branch always goes to the bottom) in the builder's layout: a node's non-leaf
    children are contiguous, in ascending slot order.  Returns its root index."""
    root = len(nodes)
    nodes.append(0)
    att.extend(rng.integers(0, 1 << 32, 2, dtype=np.uint64).tolist())
    valid = int(rng.integers(1, 256))
    if depth == 1:
        nodes[root] = valid << 8
        return root
    nonleaf = valid & int(rng.integers(0, 256))
    if nonleaf == 0:
        nonleaf = valid & -valid
    kids = [c for c in range(8) if (nonleaf >> c) & 1]
    deep = int(rng.choice(kids))
    first = len(nodes)
    # reserve the contiguous child block, then fill each child's subtree after it
    for _ in kids:
        nodes.append(0)
        att.extend([0, 0])
    for j, c in enumerate(kids):
        d = depth - 1 if c == deep else int(rng.integers(1, depth))
        sub = _rand_subtree(rng, d, nodes, att)
        # move the subtree root's descriptor into the reserved slot: point the slot at the same children
        nodes[first + j] = nodes[sub]
        att[2 * (first + j):2 * (first + j) + 2] = att[2 * sub:2 * sub + 2]
    nodes[root] = (first << 32) | (valid << 8) | nonleaf
    return root


def _pool(nodes, att):
    return SVOData(nodes=np.array(nodes, np.uint64), attachments=np.array(att, np.uint64).astype(np.uint32))


def _render_vs_oracle(torch, oracle_mod, uploads, full_nodes, full_att, cam, w=200, h=150):
    """uploads: [(SVOData, offset)] in upload order; oracle sees the combined pool."""
    osvo = oracle_mod.OracleSVO(nodes=full_nodes, attachments=full_att)
    c2w, inv_proj = cam.uniforms(w, h)
    m = RaytracingMaster(device=0, capacity_nodes=len(full_nodes))
    try:
        for data, off in uploads:
            m.SetSVOBuffer(data, offset=off)
        m.UpdateShaderParameters(cam, w, h)
        for mode in (0, 1):
            rgba, hits = m.Render(w, h, stack_mode=mode)
            ref, ref_rgba, _ = oracle_mod.render(osvo, oracle_mod.make_camera(c2w, inv_proj, (0.5, 0.5), main_light()),
                                                 w, h, mode)
            assert hits.tobytes() == ref.tobytes()
            assert rgba.reshape(-1, 4).tobytes() == ref_rgba.tobytes()
        return ref
    finally:
        m.close()


def test_dag_pool_shared_node_at_two_depths(torch, oracle_mod):
    """A shared 6-level subtree reached at depth 2 and at depth 4: the walk sees
    the shallow path first, so the pool is traced with the full stack (a stack
    sized from the shallow depth would overflow on the deep path)."""
    rng = np.random.default_rng(3)
    nodes, att = [0, 0, 0, 0], [0] * 8
    # 0: root, children 1 (slot 0) and 2 (slot 7); 1 -> S directly; 2 -> 3 -> S
    s_root = _rand_subtree(rng, 6, nodes, att)
    # S's descriptor must sit where its parents point: make a one-node block holding a copy
    nodes[0] = (1 << 32) | (0x81 << 8) | 0x81
    nodes[1] = (s_root << 32) | (0x01 << 8) | 0x01        # slot 0 -> the block starting at S
    nodes[2] = (3 << 32) | (0x80 << 8) | 0x80
    nodes[3] = (s_root << 32) | (0x40 << 8) | 0x40
    data = _pool(nodes, att)
    full = np.array(nodes, np.uint64)
    eye = np.array([20.0, 25.0, -30.0])
    ref = _render_vs_oracle(torch, oracle_mod, [(data, 0)], full, data.attachments,
                            Camera(position=tuple(eye), rotation=look_rotation(-eye)))
    assert np.count_nonzero(ref["flags"] & 1) > 100
    assert not np.any(ref["flags"] & 6)


def test_three_linked_pools(torch, oracle_mod):
    """A chain of sub-pools (the getLeaf linking of NaiveCreator.cs:156-159 /
    Clipmap.cs:153-169, generalised): pool A at 0 links into B at 5000, B into C
    at 9000; uploaded C, B, A.  Traced with the full stack, equal to the oracle."""
    rng = np.random.default_rng(5)
    def sub(depth, base):
        n, a = [], []
        _rand_subtree(rng, depth, n, a)
        arr = np.array(n, np.uint64)
        nonzero_first = (arr >> np.uint64(32)) != 0
        arr[nonzero_first] += np.uint64(base) << np.uint64(32)
        return arr, np.array(a, np.uint64).astype(np.uint32)
    c_nodes, c_att = sub(3, 9000)
    b_nodes, b_att = sub(3, 5000)
    a_nodes, a_att = sub(3, 0)
    # turn one leaf-level node of A / B into a link: a non-leaf slot pointing at the next pool's root
    def link(arr, target):
        for i in range(len(arr)):
            if (int(arr[i]) & 0xFF) == 0 and (int(arr[i]) >> 8) & 0xFF:
                arr[i] = np.uint64((target << 32) | (0x01 << 8) | 0x01)
                return
        raise AssertionError("no leaf-level node")
    link(b_nodes, 9000)
    link(a_nodes, 5000)
    full = np.zeros(9000 + len(c_nodes), np.uint64)
    full_att = np.zeros(2 * len(full), np.uint32)
    for arr, at, off in ((a_nodes, a_att, 0), (b_nodes, b_att, 5000), (c_nodes, c_att, 9000)):
        full[off:off + len(arr)] = arr
        full_att[2 * off:2 * off + len(at)] = at
    uploads = [(SVOData(nodes=c_nodes, attachments=c_att), 9000), (SVOData(nodes=b_nodes, attachments=b_att), 5000),
               (SVOData(nodes=a_nodes, attachments=a_att), 0)]
    eye = np.array([-18.0, 30.0, -26.0])
    ref = _render_vs_oracle(torch, oracle_mod, uploads, full, full_att,
                            Camera(position=tuple(eye), rotation=look_rotation(-eye)))
    assert np.count_nonzero(ref["flags"] & 1) > 100


@pytest.mark.parametrize("devices", [None, [0, 0, 0]])
def test_clipmap_linked_sub_svo_trunk_first(torch, oracle_mod, devices):
    """Clipmap.UpdateMasterOctree (Clipmap.cs:153-169): a trunk built with every
    leaf linked to descriptor 10000 (NaiveCreator.Create(root, x => 10000),
    NaiveCreator.cs:156-159; builder.link_leaves) is uploaded FIRST, then the
    sub-SVO at offset 10000 (SetSVOBuffer(data, 10000)).  Between the two uploads
    the links read the zero-filled pool (empty descriptors); after the second,
    the frame equals the oracle's over the combined pool, both stack modes, with beam
    starts (the pool's longest path gives its depth; its splat list expands the shared
    sub-SVO per position), and the beam-started walk fetches fewer nodes than the
    reference's.  With a multi-device context each upload is validated once and
    replicated to the other members device to device."""
    from raytracingtest_amd.builder import link_leaves
    from raytracingtest_amd.native_builder import build_sampler_svo
    base = 10000
    trunk = link_leaves(build_sampler_svo(4, 4), lambda *a: base)
    sub = build_sampler_svo(4, 7)
    assert trunk.format == 1 and sub.format == 1 and len(trunk) < base
    full = np.zeros(base + len(sub), np.uint64)
    full[:len(trunk)] = trunk.to_v2()
    sub_v2 = sub.to_v2().copy()
    has = (sub_v2 >> np.uint64(32)) != 0
    sub_v2[has] += np.uint64(base) << np.uint64(32)
    full[base:] = sub_v2
    full_att = np.zeros(2 * len(full), np.uint32)
    full_att[:len(trunk.attachments)] = trunk.attachments
    full_att[2 * base:] = sub.attachments
    trunk_only = full.copy()
    trunk_only[base:] = 0
    eye = np.array([26.0, 30.0, -34.0])
    cam = Camera(position=tuple(eye), rotation=look_rotation(-eye))
    w, h = 320, 200
    c2w, inv_proj = cam.uniforms(w, h)
    ocam = oracle_mod.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
    m = RaytracingMaster(device=0, capacity_nodes=len(full), devices=devices)
    try:
        m.SetSVOBuffer(trunk)
        m.UpdateShaderParameters(cam, w, h)
        _, hits0 = m.Render(w, h)
        ref0, _, _ = oracle_mod.render(oracle_mod.OracleSVO(nodes=trunk_only, attachments=full_att), ocam, w, h)
        assert hits0.tobytes() == ref0.tobytes()
        m.SetSVOBuffer(sub, offset=base)
        for mode in (0, 1):
            rgba, hits = m.Render(w, h, stack_mode=mode)
            ref, ref_rgba, _ = oracle_mod.render(oracle_mod.OracleSVO(nodes=full, attachments=full_att), ocam, w, h,
                                                 mode)
            assert hits.tobytes() == ref.tobytes()
            assert rgba.reshape(-1, 4).tobytes() == ref_rgba.tobytes()
        linked = np.count_nonzero((ref["flags"] & 1) != 0)
        assert linked > 500 and np.all(ref["parent"][(ref["flags"] & 1) != 0] >= base)
        # the linked pool (every trunk leaf sharing one sub-SVO: a DAG) has an exact
        # depth (its longest path) and a splat list expanded per position, so its primary rays get beam
        # starts (the frames above ran with them) and the walk they run fetches fewer nodes
        one = m if devices is None else m.member(0)
        assert one.info()["depth"] < 22
        starts = torch.empty(w * h, dtype=torch.float32, device="cuda")
        fetch_ref = torch.zeros(w * h, dtype=torch.int32, device="cuda")
        fetch_beam = torch.zeros(w * h, dtype=torch.int32, device="cuda")
        # the survey pose above and a grazing view across the linked cells (long walks before the hit)
        graze = Camera(position=(0.0, 2.0, -30.0), rotation=look_rotation((0.05, -0.12, 1.0)))
        for k, c in enumerate((cam, graze)):
            m.UpdateShaderParameters(c, w, h)
            c2w_k, ip_k = c.uniforms(w, h)
            ref_k, _, _ = oracle_mod.render(oracle_mod.OracleSVO(nodes=full, attachments=full_att),
                                            oracle_mod.make_camera(c2w_k, ip_k, (0.5, 0.5), main_light()), w, h)
            _, hits_k = m.Render(w, h)
            assert hits_k.tobytes() == ref_k.tobytes(), f"view {k}"
            torch.cuda.synchronize()
            one.beam_starts_device(w, h, starts.data_ptr())
            one.count_fetches_device(w, h, fetch_ref.data_ptr())
            one.set_count_beam(True)
            one.count_fetches_device(w, h, fetch_beam.data_ptr())
            one.set_count_beam(False)
            one.synchronize()
            st = starts.cpu().numpy()
            hit = (ref_k["flags"] & 1) != 0
            assert hit.sum() > 500 and np.isfinite(st[hit]).all()
            assert np.all(st[hit] <= ref_k["t"][hit] / 2048.0)   # every start at or before its hit
            f_ref, f_beam = int(fetch_ref.to(torch.int64).sum()), int(fetch_beam.to(torch.int64).sum())
            print(f"linked pool view {k}: {f_beam} fetches from the beam starts, {f_ref} from the cube entry "
                  f"({f_beam / f_ref:.3f})")
            assert f_beam < f_ref, (f_beam, f_ref)
    finally:
        m.close()


@pytest.mark.parametrize("devices", [None, [0, 0, 0]])
def test_render_progressive_matches_oracle(torch, oracle_mod, text_svo, devices):
    """svo_render_progressive = OnRenderImage end to end (RaytracingMaster.cs:55-74):
    each call renders a jittered sample, blends it into the device-resident
    accumulation frame with _Sample = currentSample (AddShader.shader:44-47) and
    returns the accumulated frame; equal to the oracle's per-sample render +
    orc_accumulate + orc_pack_rgba8, bit for bit.  A camera move restarts the
    accumulation; a size change starts from a zeroed frame."""
    from raytracingtest_amd.camera import jitter_offsets
    W, H = 96, 70
    cam = overview_camera()
    rm = RaytracingMaster(capacity_nodes=1 << 16, devices=devices)
    try:
        rm.SetSVOBuffer(text_svo)
        c2w, inv_proj = cam.uniforms(W, H)
        osvo = oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments)
        acc = np.zeros((W * H, 4), np.float32)
        offs = jitter_offsets(5)
        for n, off in enumerate(offs):
            rm.UpdateShaderParameters(cam, W, H, pixel_offset=tuple(float(v) for v in off))
            assert rm.currentSample == n
            rgba8, rgba = rm.RenderProgressive(W, H, want_rgba=True)
            _, smp, _ = oracle_mod.render(osvo, oracle_mod.make_camera(c2w, inv_proj, tuple(float(v) for v in off),
                                                                      main_light()), W, H)
            oracle_mod.accumulate(acc, np.ascontiguousarray(smp, np.float32), n)
            assert rgba.reshape(-1, 4).tobytes() == acc.tobytes(), f"sample {n}"
            assert np.array_equal(rgba8.reshape(-1), oracle_mod.pack_rgba8(acc))
        # camera moved: _currentSample = 0, the new sample replaces the frame
        rm.UpdateShaderParameters(main_camera(), W, H)
        assert rm.currentSample == 0
        _, rgba = rm.RenderProgressive(W, H, want_rgba8=False, want_rgba=True)
        mc2w, minv = main_camera().uniforms(W, H)
        _, smp, _ = oracle_mod.render(osvo, oracle_mod.make_camera(mc2w, minv, (0.5, 0.5), main_light()), W, H)
        assert rgba.reshape(-1, 4).tobytes() == np.ascontiguousarray(smp, np.float32).tobytes()
        with pytest.raises(SvoError):
            rm.RenderProgressive(W, H, want_rgba8=False, want_rgba=False)
    finally:
        rm.close()


def test_render_progressive_resize_restarts(torch, oracle_mod, text_svo):
    """a new render-target size reallocates the accumulation frame; the
    first sample after it must replace the frame (sample 0), not be blended into
    zeros with weight 1/(n+1) -- on the Python mirror (currentSample restarts) and in
    the plugin itself (a caller that keeps counting still gets the sample)."""
    cam = overview_camera()
    rm = RaytracingMaster(capacity_nodes=1 << 16)
    osvo = oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments)

    def oracle_sample(w, h):
        c2w, inv_proj = cam.uniforms(w, h)
        _, smp, _ = oracle_mod.render(osvo, oracle_mod.make_camera(c2w, inv_proj, (0.5, 0.5), main_light()), w, h)
        return np.ascontiguousarray(smp, np.float32)

    try:
        rm.SetSVOBuffer(text_svo)
        rm.UpdateShaderParameters(cam, 96, 70)
        for _ in range(3):
            rm.RenderProgressive(96, 70, want_rgba8=False, want_rgba=True)
        assert rm.currentSample == 3
        rm.UpdateShaderParameters(cam, 120, 64)
        _, rgba = rm.RenderProgressive(120, 64, want_rgba8=False, want_rgba=True)
        assert rm.currentSample == 1
        assert rgba.reshape(-1, 4).tobytes() == oracle_sample(120, 64).tobytes()
        # the C-ABI alone, with a caller that does not restart its count
        rm.UpdateShaderParameters(cam, 96, 70)
        out = np.zeros((96 * 70, 4), np.float32)
        _lib.check(_lib.lib().svo_render_progressive(rm._ctx, 96, 70, 0, 41, None, out.ctypes.data),
                   "svo_render_progressive")
        assert out.tobytes() == oracle_sample(96, 70).tobytes()
    finally:
        rm.close()


def _oracle_accumulated(oracle_mod, svo, cam, w, h, offs, acc=None, first=0):
    """The oracle's progressive frame: one render per jittered offset, blended in order
    with orc_accumulate as _Sample = first + k (AddShader.shader:44-47)."""
    c2w, inv_proj = cam.uniforms(w, h)
    osvo = oracle_mod.OracleSVO(nodes=svo.to_v2(), attachments=svo.attachments)
    acc = np.zeros((w * h, 4), np.float32) if acc is None else acc
    for k, off in enumerate(offs):
        _, smp, _ = oracle_mod.render(osvo, oracle_mod.make_camera(c2w, inv_proj, tuple(float(v) for v in off),
                                                                  main_light()), w, h)
        oracle_mod.accumulate(acc, np.ascontiguousarray(smp, np.float32), first + k)
    return acc


@pytest.mark.parametrize("n_samples", [1, 3, 8])
def test_render_samples_matches_oracle_accumulate(torch, oracle_mod, n_samples):
    """Samples in flight (svo_render_samples): S jittered samples traced in one launch
    (one wave per sample) and blended in order into the accumulation equal the oracle's S
    renders + orc_accumulate, bit for bit -- also continued from an existing accumulation
    (_Sample = first + k), with the display words and 3-byte RGB of the blended frame."""
    from raytracingtest_amd.camera import jitter_offsets
    svo = build_menger(7)
    cam = overview_camera()
    w, h = 203, 150   # neither a multiple of 8: partial tiles
    offs = jitter_offsets(2 * n_samples)
    want = _oracle_accumulated(oracle_mod, svo, cam, w, h, offs[:n_samples])
    rm = RaytracingMaster(device=0, capacity_nodes=len(svo))
    try:
        rm.SetSVOBuffer(svo)
        rm.UpdateShaderParameters(cam, w, h)
        acc = torch.zeros(w * h * 4, dtype=torch.float32, device="cuda")
        b = _bufs(torch, w * h)
        torch.cuda.synchronize()
        rm.render_samples(w, h, offs[:n_samples], 0, acc.data_ptr(), rgba8=b["rgba8"].data_ptr(),
                          rgb8=b["rgb8"].data_ptr())
        rm.synchronize()
        assert acc.cpu().numpy().tobytes() == want.tobytes(), "accumulation differs"
        assert np.array_equal(b["rgba8"].cpu().numpy().view(np.uint32), oracle_mod.pack_rgba8(want))
        assert np.array_equal(b["rgb8"].cpu().numpy().reshape(-1, 3),
                              oracle_mod.pack_rgba8(want).view(np.uint8).reshape(-1, 4)[:, :3])
        # the next S samples continue the accumulation
        want2 = _oracle_accumulated(oracle_mod, svo, cam, w, h, offs[n_samples:], acc=want.copy(), first=n_samples)
        rm.render_samples(w, h, offs[n_samples:], n_samples, acc.data_ptr())
        rm.synchronize()
        assert acc.cpu().numpy().tobytes() == want2.tobytes(), "continued accumulation differs"
    finally:
        rm.close()


@pytest.mark.parametrize("world,share", [(2, None), (4, 0.75)])
def test_render_samples_rank_parts_assemble(torch, oracle_mod, world, share):
    """The N > 1 samples-in-flight step on one GPU: every 'rank' traces S = 4 samples of
    its bands into its band accumulation (band layout; the display rank straight into the
    frame-layout accumulation) and sends the blended 3-byte RGB; svo_assemble_frame
    rebuilds the display frame, equal to orc_accumulate over the oracle's 4 whole-frame
    samples, then packed -- bit for bit, twice in a row (the second step continues)."""
    from raytracingtest_amd.camera import jitter_offsets
    from raytracingtest_amd.distributed import weighted_owner
    svo = build_menger(7)
    cam = overview_camera()
    w, h = 264, 203
    S = 4
    offs = jitter_offsets(2 * S, seed=7)
    owner = None if share is None else weighted_owner(world, share)
    deal = (lambda r: (8, r, world)) if owner is None else (lambda r: (8, r, world, owner))
    rm = RaytracingMaster(device=0, capacity_nodes=len(svo))
    try:
        rm.SetSVOBuffer(svo)
        rm.UpdateShaderParameters(cam, w, h)
        acc0 = torch.zeros(w * h * 4, dtype=torch.float32, device="cuda")   # display rank: frame layout
        frame8 = torch.zeros(w * h, dtype=torch.int32, device="cuda")
        accs, parts = [None], [None]
        for r in range(1, world):
            n = len(band_rows(h, deal(r))) * w
            accs.append(torch.zeros(max(n, 1) * 4, dtype=torch.float32, device="cuda"))
            parts.append(torch.zeros(max(n, 1) * 3, dtype=torch.uint8, device="cuda"))
        torch.cuda.synchronize()
        want = None
        for step in range(2):
            o = offs[step * S:(step + 1) * S]
            rm.render_samples(w, h, o, step * S, acc0.data_ptr(), rgba8=frame8.data_ptr(), layout=_lib.LAYOUT_FRAME,
                              band=deal(0))
            for r in range(1, world):
                rm.render_samples(w, h, o, step * S, accs[r].data_ptr(), rgb8=parts[r].data_ptr(), band=deal(r))
            rm.assemble_frame(w, h, [None] + [p.data_ptr() for p in parts[1:]], _lib.PART_RGB8,
                              rgba8=frame8.data_ptr(), skip_part=0, owner=owner)
            rm.synchronize()
            want = _oracle_accumulated(oracle_mod, svo, cam, w, h, o, acc=want, first=step * S)
            assert np.array_equal(frame8.cpu().numpy().view(np.uint32), oracle_mod.pack_rgba8(want)), f"step {step}"
    finally:
        rm.close()


def test_render_samples_errors(torch, text_svo):
    rm = RaytracingMaster(capacity_nodes=1 << 16)
    try:
        rm.SetSVOBuffer(text_svo)
        rm.UpdateShaderParameters(overview_camera(), 64, 64)
        acc = torch.zeros(64 * 64 * 4, dtype=torch.float32, device="cuda")
        with pytest.raises(SvoError):
            rm.render_samples(64, 64, np.zeros((9, 2), np.float32), 0, acc.data_ptr())   # > 8 samples
        with pytest.raises(SvoError):
            rm.render_samples(64, 64, np.zeros((0, 2), np.float32), 0, acc.data_ptr())
        with pytest.raises(SvoError):
            rm.render_samples(64, 64, np.zeros((2, 2), np.float32), 0, acc.data_ptr() + 4)   # misaligned
    finally:
        rm.close()


@pytest.mark.parametrize("devices", [None, [0, 0]])
def test_render_progressive_async_pipelined_frames(torch, oracle_mod, text_svo, devices):
    """svo_render_progressive_async returns the previous call's frame from the plugin's
    pinned slots (None first), equal to svo_render_progressive's display words for the
    same sample sequence; svo_progressive_last gives the newest; a returned view stays
    valid until the call after next; a size change restarts (None, sample 0)."""
    from raytracingtest_amd.camera import jitter_offsets
    W, H = 96, 70
    cam = overview_camera()
    offs = jitter_offsets(5, seed=11)
    c2w, inv_proj = cam.uniforms(W, H)
    osvo = oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments)
    acc = np.zeros((W * H, 4), np.float32)
    want = []
    for k, off in enumerate(offs):
        _, smp, _ = oracle_mod.render(osvo, oracle_mod.make_camera(c2w, inv_proj, tuple(float(v) for v in off),
                                                                  main_light()), W, H)
        oracle_mod.accumulate(acc, np.ascontiguousarray(smp, np.float32), k)
        want.append(oracle_mod.pack_rgba8(acc).copy())
    rm = RaytracingMaster(capacity_nodes=1 << 16, devices=devices)
    try:
        rm.SetSVOBuffer(text_svo)
        views = []
        for k, off in enumerate(offs):
            rm.UpdateShaderParameters(cam, W, H, pixel_offset=tuple(float(v) for v in off))
            if k == 0:
                assert rm.currentSample == 0
            got = rm.RenderProgressiveAsync(W, H, copy=False)
            if k == 0:
                assert got is None
            else:
                views.append((k - 1, got))
                assert np.array_equal(got.reshape(-1), want[k - 1]), f"frame {k - 1}"
            if len(views) >= 2:   # the view returned by the previous call is still intact
                j, v = views[-2]
                assert np.array_equal(v.reshape(-1), want[j]), f"frame {j} overwritten too early"
        last = rm.ProgressiveLast(W, H)
        assert np.array_equal(last.reshape(-1), want[-1])
        # the 3-byte format (TextureFormat.RGB24): a format change restarts the slots (None), then
        # each frame is the display words without their alpha; 203 x 70 leaves a 2-pixel tail
        rm.UpdateShaderParameters(cam, W, H, pixel_offset=tuple(float(v) for v in offs[0]))
        rm.currentSample = 0
        assert rm.RenderProgressiveAsync(W, H, rgb=True) is None
        rgb = rm.ProgressiveLast(W, H)
        assert rgb.shape == (H, W, 3)
        assert np.array_equal(rgb.reshape(-1, 3), want[0].view(np.uint8).reshape(-1, 4)[:, :3])
        rm.UpdateShaderParameters(cam, 64, 48)   # a new size: fresh accumulation and slots
        assert rm.RenderProgressiveAsync(64, 48) is None
        c2, i2 = cam.uniforms(64, 48)
        _, smp, _ = oracle_mod.render(osvo, oracle_mod.make_camera(c2, i2, (0.5, 0.5), main_light()), 64, 48)
        assert np.array_equal(rm.ProgressiveLast(64, 48).reshape(-1),
                              oracle_mod.pack_rgba8(np.ascontiguousarray(smp, np.float32)))
    finally:
        rm.close()


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_render_samples_multi_device(torch, oracle_mod, devices):
    """Samples in flight on a multi-device context (the Unity host driving N GPUs): every
    member blends S = 4 samples of its bands into its own band accumulation, the display
    member into the caller's frame, and the assembled display words equal the oracle's
    accumulation -- over two steps (the members' accumulations persist) and after a size
    change (fresh, zeroed accumulations)."""
    from raytracingtest_amd.camera import jitter_offsets
    svo = build_menger(7)
    cam = overview_camera()
    S = 4
    offs = jitter_offsets(2 * S, seed=3)
    rm = RaytracingMaster(devices=devices, capacity_nodes=len(svo))
    try:
        rm.SetSVOBuffer(svo)
        for (w, h) in ((200, 136), (96, 64)):
            rm.UpdateShaderParameters(cam, w, h)
            acc = torch.zeros(w * h * 4, dtype=torch.float32, device="cuda")
            frame8 = torch.zeros(w * h, dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            want = None
            for step in range(2):
                o = offs[step * S:(step + 1) * S]
                rm.render_samples(w, h, o, step * S, acc.data_ptr(), rgba8=frame8.data_ptr(), layout=_lib.LAYOUT_FRAME)
                rm.synchronize()
                want = _oracle_accumulated(oracle_mod, svo, cam, w, h, o, acc=want, first=step * S)
                assert np.array_equal(frame8.cpu().numpy().view(np.uint32), oracle_mod.pack_rgba8(want)), \
                    f"{w}x{h} step {step}"
        with pytest.raises(SvoError):   # the display words are the multi-device output
            rm.render_samples(96, 64, offs[:2], 0, acc.data_ptr(), layout=_lib.LAYOUT_FRAME)
    finally:
        rm.close()


@pytest.mark.parametrize("move_every", [1, 4])
def test_moving_camera_frames_match_oracle(torch, oracle_mod, move_every):
    """A camera that moves every frame (the interactive case, RaytracingMaster.cs:55-74): the
    dispatch order is rebuilt every move_every-th frame from older views' costs (svo_rt.hip
    launch, svo_config.move_every), then the pan stops and the held view gets its own order.  Placement
    only: every frame equals the oracle's frame for its own view, and so does the held one."""
    svo = build_menger(8)
    w, h = 320, 184
    eyes = [(4.0 * np.sin(0.05 * i), 20.0, -40.0 + 3.0 * i) for i in range(7)]
    cams = [overview_camera(e, (0.0, 0.0, 0.0)) for e in eyes]
    m = RaytracingMaster(device=0, capacity_nodes=len(svo), config={"move_every": move_every})
    try:
        m.SetSVOBuffer(svo)
        bufs = [_bufs(torch, w * h) for _ in cams]
        for cam, b in zip(cams, bufs):      # one frame per view, no host sync in between
            m.UpdateShaderParameters(cam, w, h)
            m.render_frame(w, h, hits=b["hits"].data_ptr(), rgba=b["rgba"].data_ptr())
        held = [_bufs(torch, w * h) for _ in range(3)]
        for b in held:                      # the pan stops: three frames at the last view
            m.render_frame(w, h, hits=b["hits"].data_ptr(), rgba=b["rgba"].data_ptr())
        m.synchronize()
        for cam, b in zip(cams, bufs):
            ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h)
            _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba"))
        for b in held:
            _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba"))
    finally:
        m.close()


def test_config_version1_struct_keeps_later_fields(torch):
    """svo_config is versioned by size: a version-1 caller's 128-byte struct (before beam_back_held)
    sets every field it holds and leaves the context's beam_back_held as it was; a struct larger than
    the library's is refused."""
    import ctypes
    from raytracingtest_amd import _lib
    m = RaytracingMaster(device=0, capacity_nodes=1 << 10, config={"beam_back_held": 3})
    try:
        L = _lib.lib()
        c = _lib.SvoConfig()
        c.size = ctypes.sizeof(c)
        assert L.svo_get_config(m._ctx, ctypes.byref(c)) == 0 and c.beam_back_held == 3 and c.version == 2
        c.size = 128            # a version-1 caller
        c.move_every = 7
        c.beam_back_held = 1    # past its size: not read
        assert L.svo_set_config(m._ctx, ctypes.byref(c)) == 0
        got = m.get_config()
        assert got["move_every"] == 7 and got["beam_back_held"] == 3
        big = (ctypes.c_uint8 * 256)()
        hdr = ctypes.cast(big, ctypes.POINTER(_lib.SvoConfig))
        hdr.contents.size = 256
        assert L.svo_set_config(m._ctx, hdr) != 0
        assert m.get_config() == got
    finally:
        m.close()
