"""Multi-GPU screen split for one 8-GPU node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI on
ROCm; "gloo" for the CPU tests).  The SVO is replicated per GPU (each rank
uploads or builds its own copy) and rays are independent, so the only
exchange is moving per-rank results to the display rank:

  * bands  -- one frame split into `band_rows`-row bands dealt round-robin to
              the ranks (interleaving balances sky vs terrain rows); rank 0
              gathers the hit records / RGBA bands and re-interleaves them.
  * samples -- every rank traces the whole frame at its own _PixelOffset
              jitter (RaytracingMaster.cs:35); the progressive accumulation of
              AddShader.shader:44-47 (running mean over samples) becomes one
              all-reduce of the RGBA frames.

Each rank's band buffer holds only its rows, in increasing y; band_rows()
in raytracing_master gives their global indices.
"""
import numpy as np

from .raytracing_master import band_rows

DEFAULT_BAND_ROWS = 8


def rank_band(rank, world, rows=DEFAULT_BAND_ROWS):
    """svo_band triple (band_rows, band_rank, band_count) for this rank."""
    return (rows, rank, world)


def max_band_len(height, world, rows=DEFAULT_BAND_ROWS):
    return max(len(band_rows(height, (rows, r, world))) for r in range(world))


def gather_bands(local, height, width, world, rank, elem_bytes, rows=DEFAULT_BAND_ROWS, dist=None):
    """All-gather every rank's band buffer (a uint8 torch tensor holding
    len(band_rows) * width * elem_bytes bytes, on the rank's device) and return,
    on every rank, the list of per-rank byte tensors trimmed to their true size.
    all_gather (not gather) so the same call works on RCCL and gloo."""
    import torch
    if dist is None:
        import torch.distributed as dist
    per = max_band_len(height, world, rows) * width * elem_bytes
    send = torch.zeros(per, dtype=torch.uint8, device=local.device)
    send[:local.numel()].copy_(local.reshape(-1))
    bufs = [torch.empty(per, dtype=torch.uint8, device=local.device) for _ in range(world)]
    dist.all_gather(bufs, send)
    out = []
    for r in range(world):
        n = len(band_rows(height, (rows, r, world))) * width * elem_bytes
        out.append(bufs[r][:n])
    return out


def assemble(parts, height, width, dtype, rows=DEFAULT_BAND_ROWS):
    """Re-interleave per-rank band arrays (numpy, any dtype of one pixel) into
    a [height, width] frame."""
    world = len(parts)
    frame = np.zeros((height, width), dtype)
    for r, part in enumerate(parts):
        ys = band_rows(height, (rows, r, world))
        frame[ys] = np.asarray(part).view(dtype).reshape(len(ys), width)
    return frame


def accumulate_samples(rgba, world, dist=None):
    """Running mean of the ranks' jittered RGBA samples (AddShader's
    alpha = 1/(n+1) blend over n = 0..world-1 equals the mean): in place."""
    if dist is None:
        import torch.distributed as dist
    dist.all_reduce(rgba)
    rgba.div_(float(world))
    return rgba
