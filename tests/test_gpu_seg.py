"""GPU parity of the segmented-ray form (svo_kernel.hip render_seg_kernel).

A heavy tile's rays are traced as SEG_K t-segments side by side.  The
form must give every output bit-identical to the continuous loop -- i.e. to the oracle's
IntersectSVO (NVIDIASVO.compute:57-198) -- whatever the segment starts are.  Checked here
with every tile segmented (svo_config.seg_all), with only the heavy classes (the class tables, the
form a launch uses), with arbitrary starts (seg_scramble: unordered, NaN, +-inf, outside the
cube), over consecutive frames (the starts are rebalanced from frame to frame), a moving
camera, a band of a split frame and the sparse payload's hit masks, in both stack modes.
"""
import numpy as np
import pytest

from raytracingtest_amd import RaytracingMaster
from raytracingtest_amd.builder import build_menger
from raytracingtest_amd.camera import CAMERAS, main_camera, main_light, overview_camera

from test_gpu_frame import _bufs, _check, _oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    t = pytest.importorskip("torch")
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def c3_svo():
    from bench import CONFIGS
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = CONFIGS["C3"]
    return build_sampler_svo(cfg["sampler"], cfg["max_level"], device=0)


def _frames(torch, oracle_mod, svo, cams, w, h, mode, n_frames=3, keys=None, config=None):
    m = RaytracingMaster(device=0, capacity_nodes=len(svo), config=config)
    try:
        m.SetSVOBuffer(svo)
        for cam in cams:
            m.UpdateShaderParameters(cam, w, h)
            ref_hits, ref_rgba, ref_pos, ref_vox = _oracle(oracle_mod, svo, cam, w, h, mode)
            for _ in range(n_frames):   # every frame rebalances the starts of the next one
                b = _bufs(torch, w * h)
                m.render_frame(w, h, stack_mode=mode, **{k: v.data_ptr() for k, v in b.items()
                                                         if keys is None or k in keys})
                m.synchronize()
                _check(b, oracle_mod, ref_hits, ref_rgba, ref_pos, ref_vox, keys=keys)
    finally:
        m.close()


@pytest.mark.parametrize("mode,k", [(0, 4), (1, 4), (0, 8), (1, 8)])
def test_every_tile_segmented_matches_oracle(torch, oracle_mod, text_svo, mode, k):
    """Every tile traced as K = 4 or 8 segments per ray: every output of every frame equals the oracle."""
    cfg = {"seg_all": k}
    _frames(torch, oracle_mod, text_svo, [main_camera(), overview_camera()], 256, 256, mode, config=cfg)
    _frames(torch, oracle_mod, build_menger(8), [overview_camera()], 480, 272, mode, config=cfg)


@pytest.mark.parametrize("mode,k", [(0, 4), (1, 4), (0, 8), (1, 8)])
def test_arbitrary_segment_starts_match_oracle(torch, oracle_mod, mode, k):
    """Starts that are unordered, NaN, +-inf or outside the cube (a new hash every launch):
    the records do not depend on them."""
    _frames(torch, oracle_mod, build_menger(8), [overview_camera()], 480, 272, mode, n_frames=4,
            keys=("hits", "rgba", "position", "voxel"), config={"seg_all": k, "seg_scramble": 12345})


@pytest.mark.parametrize("mode,table", [(0, 0x448), (1, 0x448), (0, 0x888)])
def test_c3_heavy_tiles_segmented_full_frame(torch, oracle_mod, c3_svo, mode, table):
    """The bench workload (C3, 1920x1080, flyover), each XCD's heaviest classes segmented as the
    launch's own rule does (the class table forced for every launch, K = 4 and 8 mixed): six
    consecutive frames, every ray equal to the oracle's."""
    w, h = 1920, 1080
    _frames(torch, oracle_mod, c3_svo, [CAMERAS["flyover"]()], w, h, mode, n_frames=6, keys=("hits", "rgba"),
            config={"seg_table_latency": table, "seg_table_issue": table, "seg_table_thin": table})


@pytest.mark.parametrize("seg_move", [1, 2])
def test_c3_segmented_moving_camera(torch, oracle_mod, c3_svo, seg_move):
    """A pan (a new view per frame: even splits by default, under seg_move 1 the starts carried
    over from the previous view), then held."""
    from raytracingtest_amd.camera import FLYOVER_EYE, FLYOVER_TARGET
    w, h = 1920, 1080
    cams = []
    for i in range(5):
        a = 0.01 * i
        eye = (FLYOVER_EYE[0] + 2.0 * np.sin(a), FLYOVER_EYE[1], FLYOVER_EYE[2] + 2.0 * (1.0 - np.cos(a)))
        cams.append(overview_camera(eye, FLYOVER_TARGET))
    _frames(torch, oracle_mod, c3_svo, cams, w, h, 0, n_frames=2, keys=("hits", "rgba"),
            config={"seg_table_issue": 0x488, "move_every": 1, "seg_move": seg_move})


@pytest.mark.parametrize("jit", [1, 2])
def test_c3_segmented_jittered_one_sample_launches(torch, oracle_mod, c3_svo, jit):
    """svo_render_samples one sample per launch (the one-sample route: the render launch with the
    blend in its store epilogue), a new jittered offset every launch, on the C3 frame whose heavy
    tiles are segmented once the order exists -- from even splits (the default), or under
    seg_jitter 1 from the starts another sub-pixel ray stored, with the segments past an earlier segment's record
    ended early: the accumulation equals the oracle's renders + orc_accumulate, bit for bit."""
    from raytracingtest_amd.camera import jitter_offsets
    from test_gpu_frame import _oracle_accumulated
    w, h = 1920, 1080
    cam = CAMERAS["flyover"]()
    offs = jitter_offsets(6)
    want = _oracle_accumulated(oracle_mod, c3_svo, cam, w, h, offs)
    m = RaytracingMaster(device=0, capacity_nodes=len(c3_svo), config={"seg_jitter": jit})
    try:
        m.SetSVOBuffer(c3_svo)
        m.UpdateShaderParameters(cam, w, h)
        acc = torch.zeros((w * h * 4,), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        for k in range(len(offs)):
            m.render_samples(w, h, offs[k:k + 1], k, acc.data_ptr())
        m.synchronize()
        assert acc.cpu().numpy().tobytes() == want.astype(np.float32).tobytes(), "accumulation differs"
    finally:
        m.close()


@pytest.mark.parametrize("mode,k", [(0, 4), (1, 4), (0, 8)])
def test_segmented_band_and_hit_masks(torch, oracle_mod, mode, k):
    """Rank 1's band of an 8-way 8-row split (the strong split's per-GPU launch), with the sparse
    payload's per-tile hit masks: records, RGB payload and masks equal the oracle's."""
    svo = build_menger(8)
    w, h = 512, 384
    cam = overview_camera()
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, svo, cam, w, h, mode)
    band = (8, 1, 8)
    ys = np.concatenate([np.arange(y0, min(y0 + 8, h)) for y0 in range(8, h, 64)])
    rows = len(ys)
    n_tiles = (w // 8) * ((rows + 7) // 8)
    want_hits = ref_hits.reshape(h, w)[ys].reshape(-1)
    want_rgba = ref_rgba.reshape(h, w, 4)[ys].reshape(-1, 4)
    hitpx = ((want_hits["flags"] & 1) != 0).reshape(rows, w)
    want_masks = np.zeros(n_tiles, np.uint64)
    for ty in range((rows + 7) // 8):
        for tx in range(w // 8):
            blk = hitpx[ty * 8:ty * 8 + 8, tx * 8:tx * 8 + 8]
            mask = 0
            for r, c in zip(*np.nonzero(blk)):   # lane (bit) = row * 8 + column of the tile
                mask |= 1 << (int(r) * 8 + int(c))
            want_masks[ty * (w // 8) + tx] = np.uint64(mask)
    m = RaytracingMaster(device=0, capacity_nodes=len(svo), config={"seg_all": k})
    try:
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(cam, w, h)
        for _ in range(3):
            b = _bufs(torch, rows * w)
            masks = torch.full((n_tiles,), -1, dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            m.render_frame(w, h, hits=b["hits"].data_ptr(), rgba=b["rgba"].data_ptr(), rgb8=b["rgb8"].data_ptr(),
                           stack_mode=mode, band=band, hitmask=masks.data_ptr())
            m.synchronize()
            _check(b, oracle_mod, want_hits, want_rgba, keys=("hits", "rgba", "rgb8"))
            assert np.array_equal(masks.cpu().numpy().view(np.uint64), want_masks), "hit masks differ"
    finally:
        m.close()


@pytest.mark.parametrize("k", [4, 8])
def test_wave_logged_segmented_launch_matches_oracle(torch, oracle_mod, text_svo, tmp_path, monkeypatch, k):
    """The wave-logged instantiation of the segmented kernel (render_seg_kernel<..., LOG = true>,
    launched only for a context created with SVO_WAVE_LOG): the same records as the oracle, and one
    log record per workgroup with entry and trace stamps (tools/band_floor.py's input)."""
    log = tmp_path / "wave_log.bin"
    monkeypatch.setenv("SVO_WAVE_LOG", str(log))   # read when the context is created
    # the log file holds the last launch; an order (and with it the segmented kernel) is in use from
    # the launch after next (the order builds on a side stream)
    _frames(torch, oracle_mod, text_svo, [main_camera()], 256, 256, 0, n_frames=4, config={"seg_all": k})
    monkeypatch.delenv("SVO_WAVE_LOG")
    rec = np.fromfile(log, np.uint32).reshape(-1, 12)
    entry = rec[:, 2]
    traced = entry != 0xFFFFFFFF
    assert traced.sum() == (256 // 8) * (256 // 8) * k   # every tile's K parts, one workgroup each
    assert ((entry[traced] >> 28) > 0).all()              # every entry a part (seg_all)
    assert (rec[traced, 8] > 0).all() and (rec[traced, 0] > 0).all() and (rec[traced, 1] >= rec[traced, 0]).all()
