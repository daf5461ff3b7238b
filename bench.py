"""Benchmark: SVO primary-ray throughput on MI355X (BASELINE.json metric
"Mrays/sec + achieved HBM GB/s, 1920x1080 primary rays, depth-10 SVO").

Workload (config C3 of BASELINE.json): a depth-10 (1024^3)
SVO built from the reference's Custom1 OpenSimplex terrain sampler
(SampleFunctions.cs:40-47, seed 7) by the native NaiveCreator restatement,
1920x1080 primary rays from the 'flyover' camera, Main.unity intrinsics and
light.  A step = one CSMain-equivalent pass: every pixel's camera ray,
IntersectSVO, hit decode, Shade, RGBA + 24-byte hit record written to HBM.
Inputs (node pool, camera) are resident before the timed region.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): one rank per
GPU, SVO replicated per GPU, each rank traces one full 1920x1080 jittered
sample per step (_PixelOffset from a seeded sequence, RaytracingMaster.cs:35):
weak scaling, no data-path collective in the step.  `--split bands` instead
splits ONE frame into 8-row bands across ranks and gathers the hit records to
rank 0 over RCCL every step (strong scaling).

roofline: algorithmic bytes per launch = sum over rays of
  8 * F (8-byte node fetches) + 8 * [hit] (attachment) + 24 (hit record) + 16 (RGBA)
with F counted per ray by the instrumented kernel; divided by the average
kernel duration from HIP events on the launch stream.  peak = 8 TB/s HBM.
cpu_baseline: the strict-IEEE C oracle (oracle/, "port") on the host cores.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
METRIC = "Mrays/sec + achieved HBM GB/s, 1920x1080 primary rays, depth-10 SVO"


# BASELINE.json configs; C3 is the metric's workload.  C1-C3
# trace in the HLSL stack mode, C4-C5 (> 2^24 nodes) in the exact one.
CONFIGS = {
    "C1": dict(width=256, height=256, max_level=7, sampler=4, camera="main", svo="sampler", stack_mode=0),
    "C2": dict(width=1920, height=1080, max_level=9, sampler=-1, camera="overview", svo="menger", stack_mode=0),
    "C3": dict(width=1920, height=1080, max_level=11, sampler=4, camera="flyover", svo="sampler", stack_mode=0),
    "C4": dict(width=3840, height=2160, max_level=13, sampler=4, camera="overview", svo="sampler", stack_mode=1),
    "C5": dict(width=7680, height=4320, max_level=14, sampler=4, camera="overview", svo="sampler", stack_mode=1),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", choices=sorted(CONFIGS), default="C3",
                   help="BASELINE.json workload; the flags below override its fields")
    p.add_argument("--width", type=int, default=None)
    p.add_argument("--height", type=int, default=None)
    p.add_argument("--max-level", type=int, default=None, help="NaiveCreator maxLevel (depth + 1)")
    p.add_argument("--sampler", type=int, default=None, help="SampleFunctions.Type (4 = Custom1)")
    p.add_argument("--stack-mode", type=int, default=None, help="0 = HLSL float2 stack, 1 = exact")
    p.add_argument("--split", choices=["samples", "bands"], default="samples")
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU-baseline time budget (0 = skip)")
    p.add_argument("--no-rgba", action="store_true")
    p.add_argument("--camera", choices=["flyover", "overview", "main"], default=None)
    p.add_argument("--shadows", action="store_true", help="C3 '+1 shadow ray' pass after the primary rays")
    p.add_argument("--accumulate", action="store_true",
                   help="samples mode: all-reduce the RGBA samples (progressive accumulation) every step")
    a = p.parse_args()
    cfg = CONFIGS[a.config]
    for k in ("width", "height", "max_level", "sampler", "camera", "stack_mode"):
        if getattr(a, k) is None:
            setattr(a, k, cfg[k])
    a.svo = cfg["svo"]
    return a


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU over RCCL; SVO_BENCH_BACKEND=gloo + ranks sharing a GPU is
    # only for rehearsing the N>1 plumbing on a one-GPU box
    backend = os.environ.get("SVO_BENCH_BACKEND", "nccl")
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from raytracingtest_amd import RaytracingMaster, band_rows
    from raytracingtest_amd.camera import CAMERAS, jitter_offsets
    from raytracingtest_amd.native_builder import build_sampler_svo

    W, H = args.width, args.height
    t0 = time.time()
    if args.svo == "menger":   # 256^3 Menger sponge surface voxels
        from raytracingtest_amd.builder import build_menger
        svo = build_menger(depth=args.max_level - 1)
    else:
        svo = build_sampler_svo(args.sampler, args.max_level, device=dev.index)
    build_s = time.time() - t0
    n_nodes = len(svo)

    rm = RaytracingMaster(device=dev.index, capacity_nodes=n_nodes)
    rm.SetSVOBuffer(svo)
    cam = CAMERAS[args.camera]()
    if args.split == "samples":
        off = (0.5, 0.5) if rank == 0 else tuple(float(v) for v in jitter_offsets(world)[rank])
        band = None
        rows = H
    else:
        off = (0.5, 0.5)
        band = (8, rank, world)
        rows = len(band_rows(H, band))   # == D.rank_band(rank, world)
    rm.UpdateShaderParameters(cam, W, H, pixel_offset=off)
    if args.shadows:
        rm.SetShadowRays(True)

    n_px = W * rows
    hits = torch.empty(n_px * 24, dtype=torch.uint8, device=dev)
    rgba = None if args.no_rgba else torch.empty(n_px * 4, dtype=torch.float32, device=dev)
    # a dedicated (non-null) stream: the kernel and the timing events share it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    from raytracingtest_amd import distributed as D
    gather = args.split == "bands" and world > 1
    accumulate = args.split == "samples" and args.accumulate and world > 1 and rgba is not None

    def step():
        rm.render_device(W, H, rgba_ptr=None if rgba is None else rgba.data_ptr(), hits_ptr=hits.data_ptr(),
                         stack_mode=args.stack_mode, band=band, stream=sptr)
        if gather:       # hit-record bands -> every rank (RCCL all_gather over xGMI)
            D.gather_bands(hits, H, W, world, rank, 24, dist=dist)
        if accumulate:   # AddShader progressive accumulation across the ranks' samples
            D.accumulate_samples(rgba, world, dist=dist)

    # instrumented pass (outside the timed region): per-ray fetch counts
    fetch = torch.zeros(n_px, dtype=torch.int32, device=dev)
    rm.count_fetches_device(W, H, fetch.data_ptr(), stack_mode=args.stack_mode, band=band, stream=sptr)
    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize(dev)
    host_hits = hits.cpu().numpy().view(np.dtype([("parent", "<u4"), ("hit_idx", "u1"), ("hit_scale", "u1"),
                                                  ("flags", "<u2"), ("t", "<f4"), ("nx", "<f4"), ("ny", "<f4"),
                                                  ("nz", "<f4")]))
    n_hit = int(np.count_nonzero(host_hits["flags"] & 1))
    F = int(fetch.to(torch.int64).sum().item())
    bytes_per_launch = 8 * F + 8 * n_hit + 24 * n_px + (0 if rgba is None else 16 * n_px)

    # timed region: K steps between barrier + synchronize.  HIP events around each
    # step only with SVO_STEP_EVENTS=1 (diagnostics): their stream markers add
    # ~8 us to every step they bracket (measured 0.1265 vs 0.1182 ms per step)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    step_events = os.environ.get("SVO_STEP_EVENTS", "0") != "0"
    for i in range(args.steps):
        if step_events:
            ev[i][0].record(stream)
        step()
        if step_events:
            ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    step_ms = float(np.mean([a.elapsed_time(b) for a, b in ev])) if step_events else None
    # the roofline's kernel time: the primary-ray kernel's own mean duration, from
    # HIP events the library records on the launch stream around that kernel
    # alone (SVO_OPT_KERNEL_TIMING), over K more steps of the same workload right
    # after the timed region (event pairs inside the timed steps would add
    # stream markers to the measured step time)
    rm.set_kernel_timing(True)
    rm.kernel_time()   # forget anything recorded before
    for i in range(args.steps):
        step()
    kern_ms, n_timed = rm.kernel_time()
    rm.set_kernel_timing(False)
    if n_timed != args.steps:
        raise RuntimeError(f"kernel timing: {n_timed} launches recorded, {args.steps} expected")
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_max = float(t[0]), float(t[1])
    else:
        kern_ms_max = kern_ms

    # C3's '+1 shadow ray' (BASELINE.json configs[2]): the same frame with the
    # shadow pass, timed separately on one GPU (reported beside, not as `value`)
    shadow = None
    if world == 1 and not args.shadows and args.svo != "menger" and args.steps > 0:
        rm.SetShadowRays(True)
        for _ in range(2):
            step()
        k = max(1, args.steps // 2)
        torch.cuda.synchronize(dev)
        t_sh = time.perf_counter()
        for _ in range(k):
            step()
        torch.cuda.synchronize(dev)
        sh_ms = (time.perf_counter() - t_sh) / k * 1e3
        rm.SetShadowRays(False)
        shadow = {"ms_per_frame": round(sh_ms, 4), "primary_rays": n_px, "shadow_rays": n_hit,
                  "Mrays_per_s": round((n_px + n_hit) / (sh_ms * 1e-3) / 1e6, 2),
                  "note": "primary pass + one shadow ray per primary hit (RaytraceCompute.compute:105-112), "
                          "whole step on the host clock between synchronizes, like value"}

    rays_per_step = n_px * world
    ms_per_step = elapsed / args.steps * 1e3
    mrays = rays_per_step / (ms_per_step * 1e-3) / 1e6
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9

    if rank == 0:
        cpu = cpu_baseline(args, svo, cam, off, host_hits) if (world == 1 and args.cpu_seconds > 0) else None
        kind = "Menger" if args.svo == "menger" else "Custom1"
        workload = (f"{args.config} depth-{args.max_level - 1} ({1 << (args.max_level - 1)}^3) {kind} SVO, "
                    f"{W}x{H} primary rays" + (" + 1 shadow ray per hit" if args.shadows else "") +
                    f", {args.camera} camera")
        # the committed PMC figure is per launch of the full-frame workload (not a band of it)
        traffic = pmc_traffic(workload) if band is None else None
        out = {
            "metric": METRIC,
            "value": round(mrays, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak" if args.split == "samples" else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic: 256^3 Menger sponge surface SVO (SURVEY.md 8(d) C2)" if args.svo == "menger" else
                     "synthetic: Custom1 OpenSimplex(seed 7) terrain SVO built on-GPU by the NaiveCreator restatement"),
            "config": {"workload": workload,
                       "svo_nodes": n_nodes, "svo_format": "V%d" % svo.format, "svo_leaves": getattr(svo, "n_leaves", None),
                       "build_s": round(build_s, 2), "stack_mode": "hlsl" if args.stack_mode == 0 else "exact",
                       "rays_per_gpu_step": n_px, "hit_fraction": round(n_hit / n_px, 4),
                       "fetches_per_ray": round(F / n_px, 3), "parallelism": f"{args.split}{world}" + ("+allreduce" if accumulate else "") + ("+allgather" if gather else "")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic,
                         "kernel_ms": round(kern_ms, 4), "kernel_ms_max_rank": round(kern_ms_max, 4),
                         "kernel": "render_tile_kernel (primary rays; library HIP events around that kernel alone, K steps after the timed region)",
                         "step_ms_events": None if step_ms is None else round(step_ms, 4),
                         "algorithmic_bytes_per_launch": bytes_per_launch,
                         "bytes_formula": "8*F + 8*hits + 24*rays + 16*rays(rgba)" +
                                          (" (primary pass only; kernel_ms covers both passes)" if args.shadows else "")},
            "cpu_baseline": cpu,
            "c3_plus_shadow_ray": shadow,
        }
        print(json.dumps(out), flush=True)
    rm.close()
    if world > 1:
        dist.destroy_process_group()


def pmc_traffic(workload):
    """HBM bytes per launch of the render kernel from the committed rocprofv3 PMC
    summary (profiles/pmc_summary.json, tools/pmc_summary.py) when it was taken
    on this same workload, else None."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    return d.get("hbm_bytes_per_launch") if d.get("workload") == workload else None


def cpu_baseline(args, svo, cam, off, gpu_hits):
    """Oracle ("port") on the host cores over rows of the same frame, bounded by
    --cpu-seconds; the rows it traces are also compared with the GPU records."""
    from oracle import oracle as orc
    from raytracingtest_amd.camera import main_light

    W, H = args.width, args.height
    threads = min(16, os.cpu_count() or 1)
    c2w, inv_proj = cam.uniforms(W, H)
    ocam = orc.make_camera(c2w, inv_proj, off, main_light())
    osvo = orc.OracleSVO(nodes=svo.to_v2(), attachments=svo.attachments)
    # calibrate on 8 rows spread over the frame, then a bounded number of rows;
    # a frame that takes less than the budget is traced repeatedly
    ys = np.linspace(0, H - 1, 8).astype(np.int64)
    pix = (ys[:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.uint32)
    t = time.perf_counter()
    orc.render_pixels(osvo, ocam, W, H, pix, args.stack_mode, nthreads=threads)
    rate = len(pix) / (time.perf_counter() - t)
    n_rows = int(min(H, max(8, rate * args.cpu_seconds / W)))
    ys = np.unique(np.linspace(0, H - 1, n_rows).astype(np.int64))
    pix = (ys[:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.uint32)
    reps, secs = 0, 0.0
    while reps == 0 or secs < args.cpu_seconds:
        t = time.perf_counter()
        hits, _, _ = orc.render_pixels(osvo, ocam, W, H, pix, args.stack_mode, nthreads=threads)
        secs += time.perf_counter() - t
        reps += 1
    a = np.frombuffer(gpu_hits[pix].tobytes(), np.uint8).reshape(-1, 24)
    b = np.frombuffer(hits.tobytes(), np.uint8).reshape(-1, 24)
    mism = int(np.count_nonzero((a != b).any(axis=1)))
    # single-thread figure on the 8 calibration rows
    ys1 = np.linspace(0, H - 1, 8).astype(np.int64)
    pix1 = (ys1[:, None] * W + np.arange(0, W, 4)[None, :]).reshape(-1).astype(np.uint32)
    t = time.perf_counter()
    orc.render_pixels(osvo, ocam, W, H, pix1, args.stack_mode, nthreads=1)
    one_core = len(pix1) / (time.perf_counter() - t) / 1e6
    return {"value": round(reps * len(pix) / secs / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{len(ys)} full rows ({len(pix)} rays) spread over the same {W}x{H} frame x {reps} passes, "
                      f"{threads} threads, {secs:.1f} s; 1-thread rate on 8 rows: {one_core:.3f} Mrays/s",
            "one_core_mrays": round(one_core, 4),
            "parity_rays_checked": int(len(pix)), "parity_rays_mismatched": mism}


if __name__ == "__main__":
    main()
