"""Multi-GPU screen split for one 8-GPU node.

Two forms share one band layout and one display-side assemble kernel:

  * one process, several GPUs -- RaytracingMaster(devices=[...]) over the
    plugin's multi-device context (svo_create_multi): the Unity host's form; the
    display GPU pulls the other GPUs' band payloads over xGMI (peer access);
  * one process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
    ROCm; "gloo" for the CPU tests) -- bench.py's form: the display rank renders
    its own bands straight into the frame, every other rank into a
    band-contiguous payload, `gather_to_root` moves those payloads to the display
    rank in one batch of RCCL sends / receives, and the display rank's plugin
    rebuilds the other ranks' rows (RaytracingMaster.assemble_frame,
    svo_assemble_frame with skip_part = the display rank).

Band layout: rows are grouped in `band_rows`-row bands dealt round-robin to the
ranks (band b -> rank b % world), so sky and terrain rows interleave and every
rank gets the same mix (the reference's single dispatch grid is split,
RaytracingMaster.cs:66-68).  A rank's payload holds only its rows, in
increasing y; band_rows() in raytracing_master gives their global indices.

Payloads: 4-byte RGBA8 display words (the framebuffer the display shows) or
12-byte compact records (svo_hit_compact) from which the display GPU rebuilds
the full 24-byte hit records and the RGBA32F Result with its own SVO replica.
"""
import math

import numpy as np

from .raytracing_master import band_rows

DEFAULT_BAND_ROWS = 8


def rank_band(rank, world, rows=DEFAULT_BAND_ROWS, owner=None):
    """svo_band deal of this rank: (band_rows, band_rank, band_count) round-robin, or
    with an owner table (weighted_owner) appended."""
    return (rows, rank, world) if owner is None else (rows, rank, world, tuple(owner))


def band_len(height, rank, world, rows=DEFAULT_BAND_ROWS, owner=None):
    return len(band_rows(height, rank_band(rank, world, rows, owner)))


def max_band_len(height, world, rows=DEFAULT_BAND_ROWS, owner=None):
    return max(band_len(height, r, world, rows, owner) for r in range(world))


def weighted_owner(world, display_share, per_round=8):
    """Owner table of a weighted deal: `per_round` rounds in which every rank but
    the display rank (0) takes one band and rank 0 takes one in only
    round(display_share * per_round) of them -- rank 0 also receives and assembles
    the frame, so it gets fewer rows.  Rounds interleave the ranks,
    so a partial cycle at the frame's bottom stays balanced.  One rank: None
    (round-robin, the whole frame) -- an empty table would read as "no owner" on
    the plugin side but divide by zero in band_rows."""
    if world <= 1:
        return None
    k = int(round(min(max(display_share, 0.0), 1.0) * per_round))
    owner = []
    for j in range(per_round):
        owner += [r for r in range(world) if r > 0 or j < k]
    return owner


def weak_frame(width, height, world):
    """Frame of a weak-scaling run on `world` GPUs: the same camera at sqrt(world)
    times the linear resolution, so every GPU traces about width * height rays
    with the same per-ray cost mix as the one-GPU frame.  Width is kept a
    multiple of 64 (whole XCD tile-column strips), height a multiple of 8."""
    if world == 1:
        return width, height
    s = math.sqrt(world)
    w = max(64, int(round(width * s / 64.0)) * 64)
    h = max(8, int(round(height * s / 8.0)) * 8)
    return w, h


def gather_parts(send, parts, dst=0, dist=None, group=None):
    """One gather of every rank's equally sized payload tensor `send` into
    `parts` (a list of world tensors on the display rank `dst`, None elsewhere).
    On RCCL (backend "nccl") the transfer runs on the communicator's stream,
    ordered after the caller's current stream; on gloo it is a CPU copy."""
    if dist is None:
        import torch.distributed as dist
    if send.is_cuda and dist.get_backend(group) == "gloo":
        # gloo gathers host tensors only: the one-GPU rehearsal of the N > 1 path
        # (tools/rehearse_ranks.sh) stages through host memory; RCCL moves device
        # memory over xGMI directly
        host = send.cpu()
        hparts = [p.cpu() for p in parts] if parts is not None else None
        dist.gather(host, gather_list=hparts, dst=dst, group=group)
        if parts is not None:
            for p, h in zip(parts, hparts):
                p.copy_(h)
        return
    dist.gather(send, gather_list=parts, dst=dst, group=group)


def gather_to_root(send, parts, root=0, dist=None, group=None):
    """The N > 1 step's gather without the root's own part: every rank but
    `root` sends its payload tensor `send` to `root`, which receives rank r's
    into parts[r] (parts[root] is unused: the display rank renders its own
    bands straight into the frame).  One batch of point-to-point transfers
    (RCCL: one ncclGroupStart/End of sends and receives over xGMI), waited for
    on the caller's current stream."""
    if dist is None:
        import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    tensors = [send] if rank != root else [p for r, p in enumerate(parts) if r != root]
    staged = dist.get_backend(group) == "gloo" and any(t is not None and t.is_cuda for t in tensors)
    ops, copies = [], []
    if rank == root:
        for r in range(world):
            if r == root:
                continue
            buf = parts[r]
            if staged:   # gloo moves host tensors only (one-GPU rehearsal)
                host = buf.cpu()
                copies.append((buf, host))
                buf = host
            ops.append(dist.P2POp(dist.irecv, buf, r, group))
    else:
        ops.append(dist.P2POp(dist.isend, send.cpu() if staged else send, root, group))
    if not ops:
        return
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    for dev_buf, host in copies:
        dev_buf.copy_(host)


def gather_fixed_to_root(send, parts, root=0, dist=None, group=None):
    """gather_to_root for equal-size payloads as ONE collective call (RCCL: the
    same ncclGroup of sends / receives, issued from C++ instead of one Python op
    per peer -- the display rank's host issues every step's calls within one
    render's time).  The root passes its own payload-sized `send` too and
    parts[root] must be that same tensor (torch copies it onto itself: a no-op)."""
    if dist is None:
        import torch.distributed as dist
    rank = dist.get_rank(group)
    if send.is_cuda and dist.get_backend(group) == "gloo":   # host staging (one-GPU rehearsal)
        host = send.cpu()
        hparts = [p.cpu() for p in parts] if rank == root else None
        dist.gather(host, gather_list=hparts, dst=root, group=group)
        if rank == root:
            for r, (p, h) in enumerate(zip(parts, hparts)):
                if r != root:
                    p.copy_(h)
        return
    dist.gather(send, gather_list=parts if rank == root else None, dst=root, group=group)


def broadcast_svo(svo, src=0, dist=None, device=None):
    """Replicate a node pool from rank `src` to every rank (the
    SVO replicated per GPU, broadcast from rank 0 over xGMI).  `svo` is the
    SVOData on `src` (ignored elsewhere); the arrays travel as device tensors in
    one RCCL broadcast each, and every rank gets an SVOData with identical
    bytes (which its plugin then validates and uploads).  On gloo (CPU tests,
    one-GPU rehearsal) host tensors are broadcast."""
    import torch
    from .svo_data import SVOData
    if dist is None:
        import torch.distributed as dist
    rank = dist.get_rank()
    on_dev = device is not None and dist.get_backend() != "gloo"
    dev = device if on_dev else "cpu"
    head = torch.zeros(4, dtype=torch.int64, device=dev)
    if rank == src:
        words = svo.childDescriptors if svo.format == 1 else svo.nodes
        head[:] = torch.tensor([svo.format, len(words), len(svo.attachments), getattr(svo, "n_leaves", -1) or -1])
    dist.broadcast(head, src)
    fmt, n, n_att, n_leaves = (int(v) for v in head.tolist())
    if rank == src:
        words = svo.childDescriptors if svo.format == 1 else svo.nodes
        w = torch.from_numpy(np.ascontiguousarray(words).view(np.int32 if fmt == 1 else np.int64)).to(dev)
        a = torch.from_numpy(np.ascontiguousarray(svo.attachments).view(np.int32)).to(dev)
    else:
        w = torch.empty(n, dtype=torch.int32 if fmt == 1 else torch.int64, device=dev)
        a = torch.empty(n_att, dtype=torch.int32, device=dev)
    dist.broadcast(w, src)
    dist.broadcast(a, src)
    if rank == src:
        return svo
    words = w.cpu().numpy()
    att = a.cpu().numpy().view(np.uint32)
    out = (SVOData(childDescriptors=words.view(np.int32), attachments=att) if fmt == 1 else
           SVOData(nodes=words.view(np.uint64), attachments=att))
    if n_leaves >= 0:
        out.n_leaves = n_leaves
    return out


def gather_bands(local, height, width, world, rank, elem_bytes, rows=DEFAULT_BAND_ROWS, dist=None):
    """Gather every rank's band buffer (uint8 tensor of band_len * width *
    elem_bytes bytes) to rank 0; returns the per-rank byte tensors trimmed to
    their true size on rank 0, None elsewhere."""
    import torch
    per = max_band_len(height, world, rows) * width * elem_bytes
    send = torch.zeros(per, dtype=torch.uint8, device=local.device)
    send[:local.numel()].copy_(local.reshape(-1))
    bufs = [torch.empty(per, dtype=torch.uint8, device=local.device) for _ in range(world)] if rank == 0 else None
    gather_parts(send, bufs, dst=0, dist=dist)
    if rank != 0:
        return None
    return [bufs[r][:band_len(height, r, world, rows) * width * elem_bytes] for r in range(world)]


def assemble(parts, height, width, dtype, rows=DEFAULT_BAND_ROWS):
    """Re-interleave per-rank band arrays (numpy, any dtype of one pixel) into
    a [height, width] frame: the host restatement of the assemble kernel's
    layout (tests)."""
    world = len(parts)
    frame = np.zeros((height, width), dtype)
    for r, part in enumerate(parts):
        ys = band_rows(height, (rows, r, world))
        frame[ys] = np.asarray(part).view(dtype).reshape(len(ys), width)
    return frame


def accumulate_samples(rgba, world, dist=None):
    """Running mean of the ranks' jittered RGBA samples (AddShader's
    alpha = 1/(n+1) blend over n = 0..world-1 equals the mean in exact
    arithmetic; in float32 the all-reduce's summation order differs from the
    sequential blend, so this is the sample-parallel replica form, not bit-exact
    with the reference's order -- svo_render_samples keeps that order bit for bit,
    DESIGN.md 6.1b): in place."""
    if dist is None:
        import torch.distributed as dist
    dist.all_reduce(rgba)
    rgba.div_(float(world))
    return rgba
