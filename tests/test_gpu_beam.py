"""GPU parity of the beam starts (svo_kernel.hip beam_splat_kernel + trace_beam).

Every primary ray of a tree pool starts at its tile's lower bound of the hit t (the distance to
the nearest box of the pool's splat list whose projection touches the tile) instead of the cube
entry, in trace_seg's exact skip form.  The records must stay bit-identical to the oracle's
IntersectSVO (NVIDIASVO.compute:57-198): checked for the survey poses, cameras inside and far
outside the cube, axis-aligned and very wide views, jittered pixel offsets at the ends of [0, 1],
the samples-in-flight launch, a band of a split frame, every splat depth from the leaves up, and
both stack modes.
"""
import numpy as np
import pytest

from raytracingtest_amd import RaytracingMaster
from raytracingtest_amd.builder import build_menger
from raytracingtest_amd.camera import CAMERAS, Camera, look_rotation, main_light, overview_camera

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


def _cams():
    return {
        "flyover": CAMERAS["flyover"](),
        "main": CAMERAS["main"](),
        "overview": CAMERAS["overview"](),
        "terrain": CAMERAS["terrain"](),
        # inside the cube below the terrain surface (the camera within a splat box: the global word)
        "buried": overview_camera((3.0, -20.0, 2.0), (0.0, -25.0, 20.0)),
        # looking straight along +z and straight down: rays parallel to an axis plane (|coef| = inf)
        "axis_z": overview_camera((0.25, 4.0, -31.0), (0.25, 4.0, 10.0)),
        "down": overview_camera((0.0, 40.0, 0.0), (0.0, -10.0, 0.5)),
        # far outside the cube, and a 160-degree view inside it
        "far": overview_camera((300.0, 200.0, -500.0), (0.0, 0.0, 0.0)),
        "wide": Camera(position=(1.0, 1.0, 1.0), fov=160.0),
    }


def _render(torch, m, w, h, mode, keys=("hits", "rgba", "position", "voxel")):
    b = _bufs(torch, w * h)
    m.render_frame(w, h, stack_mode=mode, **{k: v.data_ptr() for k, v in b.items() if k in keys})
    m.synchronize()
    return b


@pytest.mark.parametrize("mode", [0, 1])
def test_beam_starts_match_oracle_c3_poses(torch, oracle_mod, c3_svo, mode):
    """The C3 terrain pool (depth 10), nine poses, two frames each: every record equals the oracle's."""
    w, h = 640, 360
    m = RaytracingMaster(device=0, capacity_nodes=len(c3_svo))
    try:
        m.SetSVOBuffer(c3_svo)
        for name, cam in _cams().items():
            m.UpdateShaderParameters(cam, w, h)
            ref_hits, ref_rgba, ref_pos, ref_vox = _oracle(oracle_mod, c3_svo, cam, w, h, mode)
            for _ in range(2):
                b = _render(torch, m, w, h, mode)
                try:
                    _check(b, oracle_mod, ref_hits, ref_rgba, ref_pos, ref_vox, keys=("hits", "rgba", "position", "voxel"))
                except AssertionError as e:
                    raise AssertionError(f"pose {name}: {e}") from None
    finally:
        m.close()


@pytest.mark.parametrize("back", [0, 1, 4, 9])
def test_every_splat_depth_matches_oracle(torch, oracle_mod, c3_svo, back):
    """Boxes from the leaves themselves (0) up to depth 1 (9): the bound only gets looser.  The
    splat depth is set after the upload, so the context rebuilds the pool's splat list from its
    device copy (svo_set_config)."""
    w, h = 480, 270
    m = RaytracingMaster(device=0, capacity_nodes=len(c3_svo))
    try:
        m.SetSVOBuffer(c3_svo)
        m.set_config(beam_back=back)
        for name in ("flyover", "main", "buried"):
            cam = _cams()[name]
            m.UpdateShaderParameters(cam, w, h)
            ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, c3_svo, cam, w, h, 0)
            b = _render(torch, m, w, h, 0, keys=("hits", "rgba"))
            _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba"))
    finally:
        m.close()


@pytest.mark.parametrize("off", [(0.0, 0.0), (1.0, 1.0), (0.999, 0.001), (0.5, 0.5)])
def test_pixel_offsets_at_the_ends_of_the_range(torch, oracle_mod, c3_svo, off):
    """_PixelOffset anywhere in [0, 1] (RaytracingMaster.cs:35): the splat covers a tile's whole
    pixel area, so the bound holds for every offset."""
    w, h = 480, 270
    cam = CAMERAS["flyover"]()
    m = RaytracingMaster(device=0, capacity_nodes=len(c3_svo))
    try:
        m.SetSVOBuffer(c3_svo)
        m.UpdateShaderParameters(cam, w, h, pixel_offset=off)
        ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, c3_svo, cam, w, h, 0, off=off)
        b = _render(torch, m, w, h, 0, keys=("hits", "rgba"))
        _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba"))
    finally:
        m.close()


def test_beam_on_and_off_give_identical_frames(torch, c3_svo):
    """The full C3 bench frame (1920x1080, flyover and Main.unity poses): the beam-started launch and
    the continuous one write the same bytes in every output."""
    w, h = 1920, 1080
    out = {}
    for beam in (1, 0):
        m = RaytracingMaster(device=0, capacity_nodes=len(c3_svo), config={"beam": beam})
        try:
            m.SetSVOBuffer(c3_svo)
            for name in ("flyover", "main"):
                m.UpdateShaderParameters(CAMERAS[name](), w, h)
                for _ in range(3):   # the order settles; every frame must match
                    b = _render(torch, m, w, h, 0, keys=("hits", "rgba", "rgba8", "position", "voxel"))
                    out.setdefault((beam, name), []).append({k: v.cpu().numpy().tobytes() for k, v in b.items()})
        finally:
            m.close()
    for name in ("flyover", "main"):
        for on, off in zip(out[(1, name)], out[(0, name)]):
            for k in on:
                assert on[k] == off[k], f"{name}: output {k} differs with beam starts"


def test_menger_and_text_pools(torch, oracle_mod, text_svo):
    """Other trees: the C2 Menger sponge (leaves at every depth of its holes) and the reference's
    Text fixture, in both stack modes."""
    for svo, (w, h) in ((build_menger(8), (480, 272)), (text_svo, (256, 256))):
        m = RaytracingMaster(device=0, capacity_nodes=len(svo))
        try:
            m.SetSVOBuffer(svo)
            for cam in (overview_camera(), CAMERAS["main"]()):
                for mode in (0, 1):
                    m.UpdateShaderParameters(cam, w, h)
                    ref_hits, ref_rgba, ref_pos, ref_vox = _oracle(oracle_mod, svo, cam, w, h, mode)
                    b = _render(torch, m, w, h, mode)
                    _check(b, oracle_mod, ref_hits, ref_rgba, ref_pos, ref_vox,
                           keys=("hits", "rgba", "position", "voxel"))
        finally:
            m.close()


def test_beam_band_and_samples(torch, oracle_mod, c3_svo):
    """Rank 2's band of a 4-way 8-row split (global rows index the full-frame bound) and a
    four-sample launch with jittered offsets (every sample's rays share the tile bound)."""
    from test_gpu_frame import _oracle_accumulated
    w, h = 640, 360
    cam = CAMERAS["flyover"]()
    ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, c3_svo, cam, w, h, 0)
    ys = np.concatenate([np.arange(y0, min(y0 + 8, h)) for y0 in range(16, h, 32)])
    m = RaytracingMaster(device=0, capacity_nodes=len(c3_svo))
    try:
        m.SetSVOBuffer(c3_svo)
        m.UpdateShaderParameters(cam, w, h)
        b = _bufs(torch, len(ys) * w)
        m.render_frame(w, h, hits=b["hits"].data_ptr(), rgba=b["rgba"].data_ptr(), band=(8, 2, 4))
        m.synchronize()
        _check(b, oracle_mod, ref_hits.reshape(h, w)[ys].reshape(-1), ref_rgba.reshape(h, w, 4)[ys].reshape(-1, 4),
               keys=("hits", "rgba"))
        offs = np.array([[0.1, 0.9], [0.7, 0.3], [0.0, 1.0], [0.55, 0.45]], np.float32)
        acc = torch.zeros((h * w * 4,), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        m.render_samples(w, h, offs, 0, acc.data_ptr())
        m.synchronize()
        want = _oracle_accumulated(oracle_mod, c3_svo, cam, w, h, offs)
        assert acc.cpu().numpy().tobytes() == want.astype(np.float32).tobytes(), "accumulation differs"
    finally:
        m.close()


def test_views_and_held_bursts_without_host_sync(torch, oracle_mod, c3_svo):
    """Beam starts are re-splatted on the launch stream at each view change and reused while the
    view is held (svo_rt.hip launch): a sequence of view changes and held-view bursts submitted with
    no host synchronisation -- each frame into its own buffers -- must give every frame its own
    view's records (a splat racing a queued render that still reads the old bound would not)."""
    from raytracingtest_amd.camera import FLYOVER_EYE, FLYOVER_TARGET
    w, h = 640, 360
    views = []
    for i in range(4):
        a = 0.05 * i
        eye = (FLYOVER_EYE[0] + 4.0 * np.sin(a), FLYOVER_EYE[1] - 2.0 * i, FLYOVER_EYE[2] + 4.0 * (1.0 - np.cos(a)))
        views.append(overview_camera(eye, FLYOVER_TARGET))
    refs = [_oracle(oracle_mod, c3_svo, cam, w, h, 0)[:2] for cam in views]
    seq = [0, 0, 0, 1, 2, 2, 3, 0, 0, 1, 1, 1, 1, 2, 3, 3, 0]
    m = RaytracingMaster(device=0, capacity_nodes=len(c3_svo))
    try:
        m.SetSVOBuffer(c3_svo)
        outs = [_bufs(torch, w * h) for _ in seq]   # (each fill synchronises the device: all before)
        for v, b in zip(seq, outs):
            m.UpdateShaderParameters(views[v], w, h)
            m.render_frame(w, h, hits=b["hits"].data_ptr(), rgba=b["rgba"].data_ptr())
        m.synchronize()
        for k, (v, b) in enumerate(zip(seq, outs)):
            try:
                _check(b, oracle_mod, refs[v][0], refs[v][1], keys=("hits", "rgba"))
            except AssertionError as e:
                raise AssertionError(f"frame {k} (view {v}): {e}") from None
    finally:
        m.close()


def _sweep_cameras(n=64, seed=0xBEA4):
    """n seeded random cameras around the C3 cube ([-16, 16]^3 world): eyes above the terrain inside
    the cube, below it (inside solid ground), just outside a face (boxes crossing the camera plane)
    and far outside; look-at points in the cube or near-axis directions (within 1e-2..1e-5 rad of
    an axis, some exactly on it); vertical FOV 10..170 degrees; a pixel offset anywhere in [0, 1]^2
    (the ends of the range included)."""
    rng = np.random.default_rng(seed)
    cams = []
    for i in range(n):
        kind = i % 4
        if kind == 0:     # inside the cube, above the terrain
            eye = rng.uniform([-15, 2, -15], [15, 15.5, 15])
        elif kind == 1:   # inside the cube, under the terrain surface
            eye = rng.uniform([-15, -15.5, -15], [15, -6, 15])
        elif kind == 2:   # just outside a face: the nearest boxes straddle the camera plane
            eye = rng.uniform(-15, 15, 3)
            ax = rng.integers(3)
            eye[ax] = rng.choice([-1, 1]) * rng.uniform(16.0, 16.5)
        else:             # far outside
            d = rng.normal(size=3)
            eye = d / np.linalg.norm(d) * rng.uniform(40, 600)
        if rng.random() < 0.3:   # near an axis direction
            fwd = np.zeros(3)
            fwd[rng.integers(3)] = rng.choice([-1.0, 1.0])
            eps = 0.0 if rng.random() < 0.3 else 10.0 ** rng.uniform(-5, -2)
            fwd = fwd + eps * rng.normal(size=3)
            if abs(fwd[1]) > 0.99:   # LookRotation's up vector must not be parallel
                fwd[0] += 1e-3
        else:
            fwd = rng.uniform(-12, 12, 3) - eye
        fov = float(rng.uniform(10, 170))
        off = rng.random(2)
        if i % 8 == 3:
            off = np.array([float(rng.integers(2)), float(rng.integers(2))])
        cams.append((Camera(position=tuple(eye), rotation=look_rotation(fwd), fov=fov), tuple(float(v) for v in off)))
    return cams


def test_beam_bound_random_camera_sweep(torch, oracle_mod, c3_svo):
    """the beam bound's conservativeness swept once over 64 seeded random cameras
    on the C3 pool at 256x144 (eyes inside / under / just outside / far outside the cube, FOV
    10..170 degrees, boxes across the camera plane, near-axis views, offsets in [0, 1]^2), both
    stack modes: every record equals the oracle's IntersectSVO (NVIDIASVO.compute:40-54,66-69 is
    where the walk starts), and on every hit ray the start the kernel used (svo_beam_starts) is at
    or below the oracle's f32 hit t.  The minimum slack, in units of the start's rounding margin
    (2 sum|coef| + sum|bias|) 2^-20, is reported (SVO_BEAM_SWEEP_OUT=<file> writes
    the summary)."""
    import json
    import os
    w, h = 256, 144
    m = RaytracingMaster(device=0, capacity_nodes=len(c3_svo))
    starts = torch.empty(w * h, dtype=torch.float32, device="cuda")
    summary = {"cameras": 0, "rays": 0, "hit_rays": 0, "beam_rays": 0, "min_slack_margins": None,
               "min_slack_rel": None, "per_camera": []}
    try:
        m.SetSVOBuffer(c3_svo)
        for i, (cam, off) in enumerate(_sweep_cameras()):
            m.UpdateShaderParameters(cam, w, h, pixel_offset=off)
            m.beam_starts_device(w, h, starts.data_ptr())
            m.synchronize()
            st = starts.cpu().numpy().astype(np.float64)
            for mode in (0, 1):
                ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, c3_svo, cam, w, h, mode, off=off)
                b = _render(torch, m, w, h, mode, keys=("hits", "rgba"))
                try:
                    _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba"))
                except AssertionError as e:
                    raise AssertionError(f"camera {i} mode {mode} ({cam.position}, fov {cam.fov:.1f}, off {off}): {e}") from None
                hit = (ref_hits["flags"] & 1) != 0
                t_svo = ref_hits["t"].astype(np.float64) / 2048.0   # bestHit.distance = 2048 t_min, exact
                sel = hit & np.isfinite(st)
                bad = np.flatnonzero(sel & (st > t_svo))
                assert len(bad) == 0, f"camera {i} mode {mode}: {len(bad)} hit rays start past their hit"
                if mode == 0 and sel.any():
                    # the start's rounding margin per ray, from the ray setup in float64
                    c2w, ip = (np.asarray(a, np.float64) for a in cam.uniforms(w, h))
                    px = (np.arange(w * h) % w + off[0]) / w * 2 - 1
                    py = (np.arange(w * h) // w + off[1]) / h * 2 - 1
                    v = ip @ np.stack([px, py, np.zeros_like(px), np.ones_like(px)])
                    d = (c2w[:3, :3] @ v[:3]).T
                    d /= np.linalg.norm(d, axis=1, keepdims=True)
                    o = c2w[:3, 3] / 32 + 1.5
                    with np.errstate(divide="ignore"):
                        coef = 1.0 / np.abs(d)
                    margin = (2 * coef.sum(1) + (coef * o[None, :]).sum(1)) * 2.0 ** -20
                    slack = (t_svo - st)[sel] / margin[sel]
                    rel = ((t_svo - st) / t_svo)[sel]
                    mn, mr = float(np.min(slack)), float(np.min(rel))
                    summary["per_camera"].append({"eye": [round(float(x), 3) for x in cam.position],
                                                  "fov": round(cam.fov, 2), "off": off, "hit_rays": int(hit.sum()),
                                                  "beam_rays": int(sel.sum()), "min_slack_margins": round(mn, 3)})
                    summary["min_slack_margins"] = mn if summary["min_slack_margins"] is None else min(mn, summary["min_slack_margins"])
                    summary["min_slack_rel"] = mr if summary["min_slack_rel"] is None else min(mr, summary["min_slack_rel"])
                    summary["beam_rays"] += int(sel.sum())
                if mode == 0:
                    summary["hit_rays"] += int(hit.sum())
            summary["cameras"] += 1
            summary["rays"] += w * h
    finally:
        m.close()
    assert summary["cameras"] == 64 and summary["beam_rays"] > 0
    if os.environ.get("SVO_BEAM_SWEEP_OUT"):
        with open(os.environ["SVO_BEAM_SWEEP_OUT"], "w") as fh:
            json.dump(summary, fh, indent=1)
    print(f"beam sweep: {summary['beam_rays']} beam-started hit rays over {summary['cameras']} cameras, "
          f"min slack {summary['min_slack_margins']:.3f} margins ({summary['min_slack_rel']:.3e} relative)")


@pytest.mark.parametrize("mode", [0, 1])
def test_held_view_resplat_is_finer_and_exact(torch, oracle_mod, c3_svo, mode):
    """A held view re-splats once with its finer list (svo_config.beam_back_held):
    the first launch at a view starts from the moving camera's depth-8 boxes, the next ones from
    every voxel's box.  Every frame of the sequence equals the oracle's, and the walk the render runs
    (SVO_OPT_COUNT_BEAM: the held list) fetches fewer descriptors than with the held list off (-1),
    every start staying at or below its ray's hit t."""
    w, h = 480, 270
    cams = [CAMERAS["flyover"](), CAMERAS["main"]()]
    fetches = {}
    for held in (0, -1):
        m = RaytracingMaster(device=0, capacity_nodes=len(c3_svo), config={"beam_back_held": held})
        try:
            m.SetSVOBuffer(c3_svo)
            assert m.get_config()["beam_back_held"] == held
            total = 0
            for cam in cams:
                m.UpdateShaderParameters(cam, w, h)
                ref_hits, ref_rgba, _, _ = _oracle(oracle_mod, c3_svo, cam, w, h, mode)
                for _ in range(3):   # a new view (coarse), then held (the fine re-splat, then reuse)
                    b = _render(torch, m, w, h, mode, keys=("hits", "rgba"))
                    _check(b, oracle_mod, ref_hits, ref_rgba, keys=("hits", "rgba"))
                m.set_count_beam(True)
                f = torch.zeros(w * h, dtype=torch.int32, device="cuda")
                m.count_fetches_device(w, h, f.data_ptr(), stack_mode=mode)
                m.set_count_beam(False)
                starts = torch.empty(w * h, dtype=torch.float32, device="cuda")
                m.beam_starts_device(w, h, starts.data_ptr())
                m.synchronize()
                total += int(f.sum().item())
                hit = (ref_hits["flags"] & 1) != 0
                t = ref_hits["t"].astype(np.float64) / 2048.0   # bestHit.distance = 2048 t_min, exact
                s = starts.cpu().numpy().astype(np.float64)
                assert not np.any(hit & np.isfinite(s) & (s > t)), "a start past its ray's hit"
            fetches[held] = total
        finally:
            m.close()
    assert fetches[0] < fetches[-1], fetches
