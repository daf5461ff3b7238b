"""World-size-2/3 gloo tests of the multi-GPU path on CPU.

The per-rank renderer is the CPU oracle (test infrastructure) standing in for
the HIP kernel; the band layout, the payload formats (RGBA8 words, 3-byte RGB,
12-byte compact records = svo_hit prefix, the sparse hit payload with its
count-first exchange) and the one gather to rank 0
(distributed.gather_to_root, the batch of sends / receives bench.py's
Gather makes on RCCL) run as in
bench.py; the re-interleave is the host restatement of the assemble kernel's
layout.  The GPU side (band render + svo_assemble_frame, the multi-device
context) is covered by tests/test_gpu_frame.py."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.conftest import GOLDEN, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _sparse_part(hit, rgb):
    """Host restatement of the sparse band payload (svo_rt.h layout, svo_pack_hits):
    [u64 hit mask per 8x8 tile][u32 hits before each tile, then the count][3-B RGB
    of every hit pixel, tile by tile, lanes in row-major order]."""
    R, W = hit.shape
    tx, ty = -(-W // 8), -(-R // 8)
    h = np.zeros((ty * 8, tx * 8), bool)
    h[:R, :W] = hit
    c = np.zeros((ty * 8, tx * 8, 3), np.uint8)
    c[:R, :W] = rgb
    lanes = h.reshape(ty, 8, tx, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
    cols = c.reshape(ty, 8, tx, 8, 3).transpose(0, 2, 1, 3, 4).reshape(-1, 64, 3)
    masks = (lanes.astype(np.uint64) << np.arange(64, dtype=np.uint64)).sum(axis=1, dtype=np.uint64)
    cnt = lanes.sum(axis=1)
    offs = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32)
    return masks.tobytes() + offs.tobytes() + cols[lanes].tobytes()


def _sparse_unpack(raw, R, W, sky):
    """The display side (the sparse assemble): hits from the part, misses from `sky`."""
    tx, ty = -(-W // 8), -(-R // 8)
    n = tx * ty
    masks = np.frombuffer(raw[:8 * n], np.uint64)
    offs = np.frombuffer(raw[8 * n:12 * n + 4], np.uint32)
    rgb = np.frombuffer(raw[12 * n + 4:], np.uint8).reshape(-1, 3)
    assert len(rgb) == offs[-1]
    out = sky.copy()
    for y in range(R):
        for x in range(W):
            t = (y // 8) * tx + x // 8
            bit = (y % 8) * 8 + x % 8
            m = int(masks[t])
            if (m >> bit) & 1:
                k = int(offs[t]) + bin(m & ((1 << bit) - 1)).count("1")
                out[y, x] = int(rgb[k, 0]) | int(rgb[k, 1]) << 8 | int(rgb[k, 2]) << 16 | 255 << 24
    return out


def _worker(rank, world, port, mode, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as orc
    from raytracingtest_amd import SVOData, band_rows
    from raytracingtest_amd import distributed as D
    from raytracingtest_amd.camera import jitter_offsets, main_light, overview_camera
    z = np.load(os.path.join(GOLDEN, "text_svo.npz"))
    svo = SVOData.from_absolute(z["abs_child_ptr"], z["valid_mask"], z["nonleaf_mask"], z["normal_code"])
    W, H = 96, 70
    c2w, inv_proj = overview_camera().uniforms(W, H)
    osvo = orc.OracleSVO(svo.childDescriptors, svo.attachments)
    if mode in ("bands", "rgba8", "rgb8", "compact"):
        cam = orc.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
        band = D.rank_band(rank, world)
        ys = band_rows(H, band)
        pix = (ys[:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.uint32)
        hits, rgba, _ = orc.render_pixels(osvo, cam, W, H, pix, nthreads=2)
        if mode == "bands":
            local = torch.from_numpy(np.frombuffer(hits.tobytes(), np.uint8).copy())
            parts = D.gather_bands(local, H, W, world, rank, 24)
            if rank == 0:
                frame = D.assemble([p.numpy() for p in parts], H, W, orc.HIT_DTYPE)
                np.save(os.path.join(out_dir, "frame.npy"), frame)
        else:   # bench.py's Gather: equal-size int32 payload slots, sent to rank 0, which keeps its own part
            elem_b = {"rgba8": 4, "rgb8": 3, "compact": 12}[mode]
            per = (D.max_band_len(H, world) * W * elem_b + 3) // 4
            if mode == "rgba8":
                raw = orc.pack_rgba8(rgba).tobytes()
            elif mode == "rgb8":   # the display word without its alpha byte
                raw = orc.pack_rgba8(rgba).view(np.uint8).reshape(-1, 4)[:, :3].tobytes()
            else:
                raw = hits.view(np.uint8).reshape(-1, 24)[:, :12].tobytes()
            send = torch.zeros(per, dtype=torch.int32)
            send.numpy().view(np.uint8)[:len(raw)] = np.frombuffer(raw, np.uint8)
            parts = [None] + [torch.full((per,), -7, dtype=torch.int32) for _ in range(1, world)] if rank == 0 else None
            if mode == "rgba8":   # the batch of point-to-point transfers
                D.gather_to_root(None if rank == 0 else send, parts, root=0)
            else:                 # bench.py's one-call gather (the display rank's own slot a dummy)
                if rank == 0:
                    parts[0] = torch.zeros(per, dtype=torch.int32)
                D.gather_fixed_to_root(parts[0] if rank == 0 else send, parts, root=0)
            if rank == 0:
                parts[0] = send   # the display rank's own rows never leave it
                dt = {"rgba8": np.dtype(np.uint32), "rgb8": np.dtype([("rgb", "u1", 3)]),
                      "compact": np.dtype([("w", "<u4", 3)])}[mode]
                trimmed = [p.numpy().view(np.uint8)[:D.band_len(H, r, world) * W * elem_b] for r, p in enumerate(parts)]
                frame = D.assemble(trimmed, H, W, dt)
                np.save(os.path.join(out_dir, "frame.npy"), frame)
    elif mode == "sparse":   # bench.py's SparseGather protocol: counts first, then exact-size parts
        cam = orc.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
        band = D.rank_band(rank, world)
        ys = band_rows(H, band)
        pix = (ys[:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.uint32)
        hits, rgba, _ = orc.render_pixels(osvo, cam, W, H, pix, nthreads=2)
        part = _sparse_part((hits["flags"] & 1).reshape(len(ys), W) != 0,
                            orc.pack_rgba8(rgba).view(np.uint8).reshape(len(ys), W, 4)[:, :, :3])
        cnt = torch.tensor([len(part)], dtype=torch.int32)
        sizes = [torch.zeros(1, dtype=torch.int32) for _ in range(world)] if rank == 0 else None
        D.gather_to_root(None if rank == 0 else cnt, sizes, root=0)
        if rank == 0:
            bufs = [None] + [torch.full((int(sizes[r].item()),), 0xEE, dtype=torch.uint8) for r in range(1, world)]
            D.gather_to_root(None, bufs, root=0)
            _, ref_rgba, _ = orc.render(osvo, cam, W, H, nthreads=2)   # the display rank's sky for misses
            frame = orc.pack_rgba8(ref_rgba).copy().reshape(H, W)
            frame[:] = 0
            for r in range(world):
                ys_r = band_rows(H, D.rank_band(r, world))
                raw = part if r == 0 else bufs[r].numpy().tobytes()
                sky = orc.pack_rgba8(ref_rgba).reshape(H, W)[ys_r]
                frame[ys_r] = _sparse_unpack(raw, len(ys_r), W, sky)
            np.save(os.path.join(out_dir, "frame.npy"), frame)
        else:
            D.gather_to_root(torch.from_numpy(np.frombuffer(part, np.uint8).copy()), None, root=0)
    else:
        off = (0.5, 0.5) if rank == 0 else tuple(float(v) for v in jitter_offsets(world)[rank])
        cam = orc.make_camera(c2w, inv_proj, off, main_light())
        _, rgba, _ = orc.render(osvo, cam, W, H, nthreads=2)
        t = torch.from_numpy(rgba.copy())
        D.accumulate_samples(t, world)
        if rank == 0:
            np.save(os.path.join(out_dir, "accum.npy"), t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,world", [("bands", 2), ("samples", 2), ("rgba8", 2), ("rgba8", 3), ("rgb8", 3),
                                        ("compact", 3), ("sparse", 3)])
def test_gloo_ranks(tmp_path, oracle_mod, text_svo, mode, world):
    mp.spawn(_worker, args=(world, _free_port(), mode, str(tmp_path)), nprocs=world, join=True)
    from raytracingtest_amd.camera import jitter_offsets, main_light, overview_camera
    W, H = 96, 70
    c2w, inv_proj = overview_camera().uniforms(W, H)
    osvo = oracle_mod.OracleSVO(text_svo.childDescriptors, text_svo.attachments)
    if mode in ("bands", "rgba8", "rgb8", "compact", "sparse"):
        cam = oracle_mod.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
        ref, ref_rgba, _ = oracle_mod.render(osvo, cam, W, H)
        got = np.load(tmp_path / "frame.npy")
        if mode == "sparse":
            assert np.array_equal(got.reshape(-1), oracle_mod.pack_rgba8(ref_rgba))
        elif mode == "bands":
            assert got.reshape(-1).tobytes() == ref.tobytes()
        elif mode == "rgba8":
            assert np.array_equal(got.reshape(-1), oracle_mod.pack_rgba8(ref_rgba))
        elif mode == "rgb8":
            assert got.tobytes() == oracle_mod.pack_rgba8(ref_rgba).view(np.uint8).reshape(-1, 4)[:, :3].tobytes()
        else:
            assert got.tobytes() == ref.view(np.uint8).reshape(-1, 24)[:, :12].tobytes()
    else:
        acc = np.zeros((W * H, 4), np.float64)
        for r in range(world):
            off = (0.5, 0.5) if r == 0 else tuple(float(v) for v in jitter_offsets(world)[r])
            cam = oracle_mod.make_camera(c2w, inv_proj, off, main_light())
            _, rgba, _ = oracle_mod.render(osvo, cam, W, H)
            acc += rgba
        np.testing.assert_allclose(np.load(tmp_path / "accum.npy"), acc / world, rtol=1e-6, atol=1e-7)


def test_weak_frame_keeps_rays_per_gpu():
    from raytracingtest_amd.distributed import weak_frame
    assert weak_frame(1920, 1080, 1) == (1920, 1080)
    assert weak_frame(1920, 1080, 4) == (3840, 2160)
    for n in (2, 3, 4, 5, 8):
        w, h = weak_frame(1920, 1080, n)
        assert w % 64 == 0 and h % 8 == 0
        assert abs(w * h / n / (1920 * 1080) - 1.0) < 0.02


def test_band_helpers_cover_frame():
    from raytracingtest_amd import band_rows
    from raytracingtest_amd.distributed import assemble, max_band_len
    for H, world in ((1080, 8), (1080, 3), (70, 2), (5, 4)):
        seen = np.concatenate([band_rows(H, (8, r, world)) for r in range(world)])
        assert np.array_equal(np.sort(seen), np.arange(H))
        assert max_band_len(H, world) == max(len(band_rows(H, (8, r, world))) for r in range(world))
    parts = [np.arange(len(band_rows(20, (8, r, 2))) * 3, dtype=np.int32) + 1000 * r for r in range(2)]
    f = assemble(parts, 20, 3, np.int32)
    assert f.shape == (20, 3) and f[0, 0] == 0 and f[8, 0] == 1000


def test_weighted_deal_covers_frame_and_balances():
    """Weighted band deal (the display rank takes fewer bands): every row owned
    exactly once, the display rank's share follows display_share, the other ranks
    stay within one band of each other, also across a partial last cycle."""
    from raytracingtest_amd import band_rows
    from raytracingtest_amd.distributed import band_len, max_band_len, rank_band, weighted_owner
    for world, share in ((2, 0.9), (4, 0.75), (8, 0.6), (8, 0.0), (3, 1.0)):
        owner = weighted_owner(world, share)
        assert len(owner) <= 256 and set(owner) <= set(range(world))
        assert owner.count(0) == round(share * 8) and all(owner.count(r) == 8 for r in range(1, world))
        for H in (1080, 3056, 4320, 37):
            seen = np.concatenate([band_rows(H, rank_band(r, world, 8, owner)) for r in range(world)])
            assert np.array_equal(np.sort(seen), np.arange(H))
            lens = [band_len(H, r, world, 8, owner) for r in range(world)]
            assert max(lens[1:]) - min(lens[1:]) <= 8
            assert max_band_len(H, world, 8, owner) == max(lens)
            if H >= 1080 and share > 0:
                assert abs(lens[0] / lens[1] - round(share * 8) / 8) < 0.15
    assert weighted_owner(3, 1.0) == [0, 1, 2] * 8


def _bcast_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from raytracingtest_amd import SVOData
    from raytracingtest_amd import distributed as D
    from raytracingtest_amd.builder import build_menger
    z = np.load(os.path.join(GOLDEN, "text_svo.npz"))
    v1 = SVOData.from_absolute(z["abs_child_ptr"], z["valid_mask"], z["nonleaf_mask"], z["normal_code"])
    v2 = build_menger(5)
    for name, src in (("v1", v1), ("v2", v2)):
        got = D.broadcast_svo(src if rank == 0 else None, 0)
        assert got.format == src.format and len(got) == len(src)
        words = got.childDescriptors if got.format == 1 else got.nodes
        ref = src.childDescriptors if src.format == 1 else src.nodes
        np.save(os.path.join(out_dir, f"{name}_{rank}.npy"),
                np.concatenate([np.frombuffer(words.tobytes(), np.uint8), np.frombuffer(got.attachments.tobytes(), np.uint8)]))
        assert words.tobytes() == ref.tobytes() and got.attachments.tobytes() == src.attachments.tobytes()
    dist.barrier()
    dist.destroy_process_group()


def test_svo_broadcast_replicas_identical(tmp_path):
    """bench.py's default replica: rank 0's node pool and
    attachments broadcast to every rank arrive byte-identical, V1 and V2."""
    world = 3
    mp.spawn(_bcast_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for name in ("v1", "v2"):
        blobs = [np.load(tmp_path / f"{name}_{r}.npy").tobytes() for r in range(world)]
        assert blobs[1] == blobs[0] and blobs[2] == blobs[0]


def test_weighted_owner_one_rank_is_round_robin():
    """with one rank the owner table would be empty (plugin: round-robin,
    band_rows: a division by zero); it is None (round-robin) instead."""
    from raytracingtest_amd import band_rows
    from raytracingtest_amd.distributed import band_len, rank_band, weighted_owner
    for share in (0.0, 0.03, 0.5, 1.0):
        owner = weighted_owner(1, share)
        assert owner is None
        assert np.array_equal(band_rows(37, rank_band(0, 1, 8, owner)), np.arange(37))
        assert band_len(1080, 0, 1, owner=owner) == 1080


class _FakeDist:
    """torch.distributed stand-in that records which collective each helper
    issues, on which backend, and the tensors it hands over."""

    def __init__(self, backend, rank, world):
        self.backend, self.rank, self.world, self.calls = backend, rank, world, []

    def get_backend(self, group=None):
        return self.backend

    def get_rank(self, group=None):
        return self.rank

    def get_world_size(self, group=None):
        return self.world

    def gather(self, t, gather_list=None, dst=0, group=None):
        self.calls.append(("gather", t, gather_list))

    def broadcast(self, t, src, group=None):
        self.calls.append(("broadcast", t, None))


class _DevTensor:
    """A tensor that claims to live on a GPU (no GPU in the CPU suite): any host
    staging (.cpu()) of it fails the test."""
    is_cuda = True

    def cpu(self):
        raise AssertionError("a device tensor was staged through the host on the RCCL branch")


def test_rccl_branch_chosen_for_device_tensors():
    """under backend "nccl" (= RCCL) the payload gather hands the
    device tensors themselves to ONE dist.gather (no host staging) and the SVO
    broadcast builds its tensors on the rank's device; under gloo the same
    helpers stage through host tensors."""
    import torch
    from raytracingtest_amd import distributed as D
    send, parts = _DevTensor(), [_DevTensor(), _DevTensor()]
    fd = _FakeDist("nccl", 0, 2)
    D.gather_fixed_to_root(send, parts, root=0, dist=fd)
    assert [c[0] for c in fd.calls] == ["gather"]
    assert fd.calls[0][1] is send and fd.calls[0][2] is parts
    fd = _FakeDist("nccl", 1, 2)
    D.gather_fixed_to_root(send, None, root=0, dist=fd)
    assert fd.calls[0][1] is send and fd.calls[0][2] is None
    fd = _FakeDist("nccl", 0, 2)
    D.gather_parts(send, parts, dst=0, dist=fd)
    assert fd.calls[0][1] is send
    # gloo + a device tensor: host staging (the one-GPU rehearsal path) is taken
    fd = _FakeDist("gloo", 1, 2)
    with pytest.raises(AssertionError, match="staged through the host"):
        D.gather_fixed_to_root(_DevTensor(), None, root=0, dist=fd)
    # broadcast_svo: on nccl its tensors live on the device it is given (here a stand-in
    # device, "meta": the header's .tolist() would need data, so stop at the first call)
    fd = _FakeDist("nccl", 1, 2)

    class _Stop(Exception):
        pass

    def bcast(t, src, group=None):
        fd.calls.append(("broadcast", t, None))
        raise _Stop()
    fd.broadcast = bcast
    with pytest.raises(_Stop):
        D.broadcast_svo(None, 0, dist=fd, device=torch.device("meta"))
    assert fd.calls[0][1].device.type == "meta"
    fd = _FakeDist("gloo", 1, 2)
    fd.broadcast = bcast
    with pytest.raises(_Stop):
        D.broadcast_svo(None, 0, dist=fd, device=torch.device("meta"))
    assert fd.calls[-1][1].device.type == "cpu"
