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
GPU, the SVO replicated per GPU (each rank builds the same bytes on its GPU),
the frame split into 8-row bands dealt round-robin to the ranks (SURVEY.md
8(e)), and every step ends with the north-star gather: rank 0 (the display
GPU) renders its own bands straight into the display frame, every other rank's
3-byte RGB band payload goes to rank 0 over RCCL (one batch of sends / receives)
and rank 0's plugin writes their rows into the frame (svo_assemble_frame).  The
gather of frame k overlaps the render of frame k+1 (two streams, double-buffered
payloads).  `value` is the configured frame split over the N GPUs (strong
scaling: for C3 the metric's own 1920x1080 frame, the reference's one dispatch
grid cut into bands, RaytracingMaster.cs:66-68); for C1-C3 the weak frame (the
same camera at sqrt(N) times the linear resolution, ~1920x1080 rays per GPU) is
measured in the same run and reported beside it as multi_gpu.other_frame.
Every rank writes the N = 1 step's per-pixel outputs (hit record + RGBA32F) for
its own pixels plus its band payload.  Strong scaling of the 1080p frame is
capped by its heaviest wave.  Without torchrun, --gpus N > 1
drives N GPUs from one process through the plugin's multi-device context (the
Unity host's form).

roofline: algorithmic bytes per launch = sum over rays of
  8 * F (8-byte V2 node fetches) + 8 * [hit] (attachment) + 24 (hit record) + 16 (RGBA)
with F counted per ray by the instrumented kernel; divided by the render
kernel's mean duration from HIP events on its launch stream.  peak = 8 TB/s HBM.
The kernel is bound by its dependent node-fetch chain (latency), not by HBM:
`bound` says so and `hbm_frac` gives the PMC-measured fabric bytes' fraction.
cpu_baseline: the strict-IEEE C oracle (oracle/, "port") on the host cores.
"""
import argparse
import ctypes
import json
import math
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
L2_PEAK_GBS = 34500.0        # MI355X_MICROARCH.md "L2 (per XCD)": aggregate L2 bandwidth
METRIC = "Mrays/sec + achieved HBM GB/s, 1920x1080 primary rays, depth-10 SVO"


# BASELINE.json configs; C3 is the metric's workload.  C1-C3
# trace in the HLSL stack mode, C4-C5 (> 2^24 nodes) in the exact one.
# gpus: the GPU count the config is defined on (C4: 4, C5: 8); per-GPU configs
# (gpus 1) scale their frame with the GPU count (weak scaling).
CONFIGS = {
    "C1": dict(width=256, height=256, max_level=7, sampler=4, camera="main", svo="sampler", stack_mode=0, gpus=1),
    "C2": dict(width=1920, height=1080, max_level=9, sampler=-1, camera="overview", svo="menger", stack_mode=0, gpus=1),
    "C3": dict(width=1920, height=1080, max_level=11, sampler=4, camera="flyover", svo="sampler", stack_mode=0, gpus=1),
    "C4": dict(width=3840, height=2160, max_level=13, sampler=4, camera="overview", svo="sampler", stack_mode=1, gpus=4),
    "C5": dict(width=7680, height=4320, max_level=14, sampler=4, camera="overview", svo="sampler", stack_mode=1, gpus=8),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None, help="GPUs (default: WORLD_SIZE under torchrun, else 1)")
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--config", choices=sorted(CONFIGS), default="C3",
                   help="BASELINE.json workload; the flags below override its fields")
    p.add_argument("--width", type=int, default=None)
    p.add_argument("--height", type=int, default=None)
    p.add_argument("--max-level", type=int, default=None, help="NaiveCreator maxLevel (depth + 1)")
    p.add_argument("--sampler", type=int, default=None, help="SampleFunctions.Type (4 = Custom1)")
    p.add_argument("--stack-mode", type=int, default=None, help="0 = HLSL float2 stack, 1 = exact")
    p.add_argument("--frame-scaling", choices=["weak", "strong"], default=None,
                   help="N > 1: strong (default) = the configured frame split over the GPUs (C3: the metric's "
                        "1920x1080 frame); weak = the frame grows with sqrt(N) per axis.  C1-C3 report the other "
                        "one beside value, labelled")
    p.add_argument("--payload", choices=["auto", "rgb8", "rgba8", "compact", "sparse"], default="auto",
                   help="N > 1: what moves to the display rank: 3-byte RGB (the display word without its "
                        "constant alpha), sparse (tile hit masks + the RGB of hit pixels only; rank 0 computes "
                        "the sky), RGBA8 display words (4 B/px) or compact records (12 B/px, rank 0 rebuilds hit "
                        "records + Result); auto (default): rgb8 or sparse, whichever ran the pipelined step "
                        "faster in a calibration run (both reported)")
    p.add_argument("--devices", default=None,
                   help="one-process multi-device mode: comma-separated HIP device indices of the context's members "
                        "(default 0..N-1; an index may repeat to rehearse the split on one GPU)")
    p.add_argument("--replica", choices=["broadcast", "build"], default="broadcast",
                   help="N ranks: the SVO built on rank 0 and broadcast over RCCL (default), or built on every rank")
    p.add_argument("--display-share", type=float, default=None,
                   help="N > 1: the display rank's share of a normal rank's bands (default: calibrated from its "
                        "assemble time; 1 = round-robin)")
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU-baseline time budget (0 = skip)")
    p.add_argument("--no-rgba", action="store_true")
    p.add_argument("--camera", choices=["flyover", "overview", "main", "terrain"], default=None)
    p.add_argument("--shadows", action="store_true", help="C3 '+1 shadow ray' pass after the primary rays")
    p.add_argument("--no-extras", "--no-extra-poses", dest="extras", action="store_false",
                   help="N = 1: skip the figures reported beside value (other camera poses, frames in flight, "
                        "host path); profiling runs use it so every render_tile_kernel launch is the value's "
                        "workload, one frame at a time")
    p.add_argument("--set", action="append", default=[], metavar="FIELD=VALUE",
                   help="svo_config field for the context (include/svo_rt.h; A/B runs): the policy only, every "
                        "setting renders the same frames")
    a = p.parse_args()
    a.svo_config = {}
    for kv in a.set:
        k, v = kv.split("=", 1)
        a.svo_config[k] = float(v) if "." in v else int(v, 0)
    cfg = CONFIGS[a.config]
    for k in ("width", "height", "max_level", "sampler", "camera", "stack_mode"):
        if getattr(a, k) is None:
            setattr(a, k, cfg[k])
    a.svo = cfg["svo"]
    a.cfg_gpus = cfg["gpus"]
    return a


def host_cpu_info():
    """CPU model, sockets, logical CPUs and the CPUs this job may use (affinity
    and cgroup quota): the cpu_baseline runs on all of the latter."""
    info = {"model": platform.processor() or None, "logical_cpus": os.cpu_count()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "Model name":
                info["model"] = v
            elif k == "Socket(s)":
                info["sockets"] = int(v)
            elif k == "Core(s) per socket":
                info["cores_per_socket"] = int(v)
            elif k == "Thread(s) per core":
                info["threads_per_core"] = int(v)
    except (OSError, ValueError, subprocess.SubprocessError):
        pass
    avail = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    info["affinity_cpus"] = avail
    info["cgroup_cpu_quota"] = quota
    info["usable_cpus"] = max(1, min(avail, int(math.floor(quota)) if quota else avail))
    return info


def main():
    args = parse()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is None:
        args.gpus = world_env
    if world_env > 1 and args.gpus != world_env:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but torchrun started WORLD_SIZE={world_env} ranks")
    mode = "ranks" if world_env > 1 else ("multidevice" if args.gpus > 1 else "single")
    import torch
    args.device_list = ([int(d) for d in args.devices.split(",")] if args.devices else list(range(args.gpus)))
    if mode == "multidevice" and len(args.device_list) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but --devices names {len(args.device_list)} devices")
    need = max(args.device_list) + 1 if mode == "multidevice" else 1
    if torch.cuda.device_count() < need:
        raise SystemExit(f"bench.py: {args.gpus} GPUs requested, {torch.cuda.device_count()} visible")
    world = args.gpus
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch.distributed as dist
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if mode == "ranks":
        # one rank per GPU over RCCL; SVO_BENCH_BACKEND=gloo + ranks sharing a GPU is
        # only for rehearsing the N>1 plumbing on a one-GPU box
        backend = os.environ.get("SVO_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from raytracingtest_amd import RaytracingMaster, _lib
    from raytracingtest_amd import distributed as D
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo

    W, H = args.width, args.height
    # N > 1: the configured frame split over the GPUs (strong scaling -- for C3 the
    # metric's own 1920x1080 frame, north_star "reported at 1, 2, 4 and 8 GPUs"); the
    # weak frame is reported beside it, labelled (measure_frame's `other`)
    scaling = args.frame_scaling or "strong"
    if world > 1 and scaling == "weak":
        W, H = D.weak_frame(W, H, world)
    t0 = time.time()
    svo = None
    if mode != "ranks" or args.replica == "build" or rank == 0:
        if args.svo == "menger":   # 256^3 Menger sponge surface voxels
            from raytracingtest_amd.builder import build_menger
            svo = build_menger(depth=args.max_level - 1)
        else:
            svo = build_sampler_svo(args.sampler, args.max_level, device=dev.index)
    build_s = time.time() - t0
    if mode == "ranks" and args.replica == "broadcast":
        # the SVO replicated per GPU from rank 0 over RCCL; each rank's
        # plugin validates and uploads its copy
        svo = D.broadcast_svo(svo, 0, device=dev)
    n_nodes = len(svo)
    cam = CAMERAS[args.camera]()

    if mode == "multidevice":
        return bench_multidevice(args, svo, cam, W, H, scaling, build_s)

    rm = RaytracingMaster(device=dev.index, capacity_nodes=n_nodes, config=args.svo_config)
    rm.SetSVOBuffer(svo)
    rm.UpdateShaderParameters(cam, W, H)
    if args.shadows:
        rm.SetShadowRays(True)
    # a dedicated (non-null) stream: the kernel and the timing events share it
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    preflight = rank_preflight(args, rank, world, dev, dist) if world > 1 else None

    m = measure_frame(args, rm, W, H, rank, world, dev, stream, dist)
    gather, hits, rgba, n_px, n_hit, F, host_hits = (m["gather"], m["hits"], m["rgba"], m["n_px"], m["n_hit"],
                                                      m["F"], m["host_hits"])
    band, deal_info, payload_choice = m["band"], m["deal_info"], m["payload_choice"]
    bytes_per_launch, elapsed, kern_ms, kern_ms_max = (m["bytes_per_launch"], m["elapsed"], m["kern_ms"],
                                                       m["kern_ms_max"])
    stages, frame_check, per_rank, step_ms = m["stages"], m["frame_check"], m["per_rank"], m["step_ms"]
    F_ref = m["F_ref"]

    # the other frame of an N > 1 run, reported beside `value` and labelled: the
    # weak frame (sqrt(N) x the linear resolution, ~W x H rays per GPU) when the run
    # is the metric's strong split, and vice versa
    other = None
    if world > 1 and args.extras and args.cfg_gpus == 1:
        other_scaling = "weak" if scaling == "strong" else "strong"
        Wo, Ho = D.weak_frame(args.width, args.height, world) if other_scaling == "weak" else (args.width, args.height)
        gather.release()
        rm.UpdateShaderParameters(cam, Wo, Ho)
        mo = measure_frame(args, rm, Wo, Ho, rank, world, dev, stream, dist)
        rm.UpdateShaderParameters(cam, W, H)
        if rank == 0:
            ms_o = mo["elapsed"] / args.steps * 1e3
            other = {"scaling": other_scaling, "frame": f"{Wo}x{Ho}", "rays_per_step": Wo * Ho,
                     "value": round(Wo * Ho / (ms_o * 1e-3) / 1e6, 2), "unit": "Mrays/s",
                     "ms_per_step": round(ms_o, 4), "steps": args.steps,
                     "rays_per_gpu_step_rank0": mo["n_px"],
                     "kernel_ms_rank0": round(mo["kern_ms"], 4), "kernel_ms_max_rank": round(mo["kern_ms_max"], 4),
                     "roofline_rank0": {"achieved": round(mo["bytes_per_launch"] / (mo["kern_ms"] * 1e-3) / 1e9, 1),
                                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                        "frac": round(mo["bytes_per_launch"] / (mo["kern_ms"] * 1e-3) / 1e9
                                                      / HBM_PEAK_GBS, 5),
                                        "algorithmic_bytes_per_launch": mo["bytes_per_launch"]},
                     "payload": mo["gather"].payload, "display_rank_deal": mo["deal_info"],
                     "per_rank_kernel_gather_assemble_ms": mo["per_rank"],
                     "assembled_frame_check": mo["frame_check"],
                     "note": ("same per-pixel outputs as value (24-B hit record + RGBA32F + the band payload); "
                              "the weak frame grows with N so every GPU traces ~1920x1080 rays -- a different "
                              "workload from the metric's 1920x1080 frame" if other_scaling == "weak" else
                              "the configured frame split over the N GPUs")}
        mo["gather"].release()
        gather = m["gather"] = None
        torch.cuda.synchronize(dev)

    # samples in flight across the ranks: S jittered samples of the same
    # frame per step, reported beside value (which stays the one-sample strong split)
    samples_n = None
    if world > 1 and args.extras and not args.shadows and args.steps > 0:
        if m["gather"] is not None:
            m["gather"].release()
            gather = m["gather"] = None
        rm.UpdateShaderParameters(cam, W, H)
        samples_n = {"frame": f"{W}x{H}", "per_samples": [measure_samples(args, rm, W, H, rank, world, dev, stream,
                                                                          dist, S) for S in (1, 2, 4, 8)],
                     "outputs": "every rank: RGBA32F accumulation of its rows + the blended band's display words "
                                "(rank 0) or 3-byte RGB payload (ranks 1..N-1, gathered once per S samples)",
                     "note": "value is the one-sample strong split; this line traces S jittered samples of the same "
                             "frame per step (svo_render_samples), rays = S x W x H per step"}

    # C3's '+1 shadow ray' (BASELINE.json configs[2]): the same frame with the
    # shadow pass, timed separately on one GPU (reported beside, not as `value`)
    shadow = None
    if world == 1 and not args.shadows and args.svo != "menger" and args.steps > 0:
        rm.SetShadowRays(True)
        for _ in range(2):
            m["step"]()
        k = max(1, args.steps // 2)
        torch.cuda.synchronize(dev)
        t_sh = time.perf_counter()
        for _ in range(k):
            m["step"]()
        torch.cuda.synchronize(dev)
        sh_ms = (time.perf_counter() - t_sh) / k * 1e3
        rm.SetShadowRays(False)
        shadow = {"ms_per_frame": round(sh_ms, 4), "primary_rays": n_px, "shadow_rays": n_hit,
                  "Mrays_per_s": round((n_px + n_hit) / (sh_ms * 1e-3) / 1e6, 2),
                  "note": "primary pass + one shadow ray per primary hit (RaytraceCompute.compute:105-112), "
                          "whole step on the host clock between synchronizes, like value"}
    host_path = host_path_rates(rm, W, H, args) if world == 1 and args.steps > 0 and args.extras else None
    in_flight = frames_in_flight(rm, W, H, args, dev) if world == 1 and args.steps > 0 and args.extras else None
    samples = (samples_in_flight(rm, W, H, args, dev, stream, floor_ms=m["floor_ms"])
               if world == 1 and args.steps > 0 and args.extras and not args.shadows else None)
    split = (strong_split_bands(rm, W, H, args, dev, stream, hits, rgba, kern_ms, m["floor_ms"])
             if world == 1 and args.steps > 0 and args.extras and not args.shadows else None)
    dropin = pan = None
    if world == 1 and args.steps > 0 and args.extras and not args.shadows:
        dropin, pan = dropin_loop_rates(rm, W, H, args, dev, stream)
    poses = None
    if world == 1 and args.extras and args.svo != "menger":
        poses = extra_poses(rm, args, W, H, hits, rgba, sptr, dev)

    rays_per_step = W * H
    ms_per_step = elapsed / args.steps * 1e3
    mrays = rays_per_step / (ms_per_step * 1e-3) / 1e6
    achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9

    if rank == 0:
        cpu = cpu_baseline(args, svo, cam, host_hits) if (world == 1 and args.cpu_seconds > 0) else None
        kind = "Menger" if args.svo == "menger" else "Custom1"
        workload = (f"{args.config} depth-{args.max_level - 1} ({1 << (args.max_level - 1)}^3) {kind} SVO, "
                    f"{W}x{H} primary rays" + (" + 1 shadow ray per hit" if args.shadows else "") +
                    f", {args.camera} camera")
        from raytracingtest_amd.build import source_digest
        digest = source_digest()
        pmc = pmc_traffic(workload, digest) if band is None else None
        traffic = pmc["hbm_bytes_per_launch"] if pmc else None
        weighted = bool(deal_info and deal_info["cycle_bands"])
        par = ("single" if world == 1 else
               f"bands{world}x8rows{'-weighted' if weighted else ''}+rccl_gather({args.payload})")
        out = {
            "metric": METRIC,
            "value": round(mrays, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic: 256^3 Menger sponge surface SVO (SURVEY.md 8(d) C2)" if args.svo == "menger" else
                     "synthetic: Custom1 OpenSimplex(seed 7) terrain SVO built on-GPU by the NaiveCreator restatement"),
            "config": {"workload": workload, "svo_config": args.svo_config or "defaults",
                       "svo_nodes": n_nodes, "svo_format": "V%d" % svo.format, "svo_leaves": getattr(svo, "n_leaves", None),
                       "build_s": round(build_s, 2), "stack_mode": "hlsl" if args.stack_mode == 0 else "exact",
                       "svo_replica": None if world == 1 else ("rccl_broadcast_from_rank0" if args.replica == "broadcast"
                                                               else "built_on_every_rank"),
                       "rays_per_step": rays_per_step, "rays_per_gpu_step": n_px,
                       "hit_fraction_rank0": round(n_hit / n_px, 4),
                       "fetches_per_ray_rank0": round(F / n_px, 3),
                       "fetches_per_ray_reference_rank0": round(F_ref / n_px, 3), "parallelism": par},
            "roofline": {"bound": "latency", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic,
                         "hbm_frac": None if traffic is None else round(traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                         "l2_frac": round(achieved / L2_PEAK_GBS, 5),
                         "kernel_ms": round(kern_ms, 4), "kernel_ms_max_rank": round(kern_ms_max, 4),
                         "kernel_ms_events": round(m["kern_ms_events"], 4),
                         "event_floor_ms": round(m["floor_ms"], 4),
                         "kernel_ms_bracket_minus_floor": round(m["kern_ms_bracket"], 4),
                         "gpu_span_ms_per_step": round(m["span_ms"], 4),
                         "kernel_ms_le_step": bool(kern_ms <= ms_per_step),
                         "kernel": "render_seg_kernel / render_tile_kernel (the primary-ray launch). N = 1: kernel_ms = "
                                   "the timed region's GPU span per launch (one HIP event pair around launches 2..K on "
                                   "their stream, from the end of the first so the host's first-launch latency is not "
                                   "in it; they run back to back and nothing else runs there at a held view); "
                                   "kernel_ms_events: library events around each launch (K more steps), which add the "
                                   "bracket's marker processing; N > 1: kernel_ms = kernel_ms_events - event_floor_ms",
                         "bound_note": "dependent node-fetch chain at 8 waves/SIMD (DESIGN.md 5.1); frac is the "
                                       "metric's algorithmic-bytes fraction of HBM peak, hbm_frac the PMC fabric "
                                       "bytes' (FETCH_SIZE x2 + WRITE_SIZE), l2_frac algorithmic bytes vs L2 peak",
                         "step_ms_events": None if step_ms is None else round(step_ms, 4),
                         "algorithmic_bytes_per_launch": bytes_per_launch,
                         "bytes_formula": "8*F + 8*hits + 24*rays + 16*rays(rgba)" +
                                          (" + payload" if world > 1 else "") +
                                          " (8 = the V2 node width; 4-byte reference descriptors would give 4*F)" +
                                          (" (primary pass only; kernel_ms covers both passes)" if args.shadows else ""),
                         # the same launch under the other accountings: node and
                         # attachment reads only, and the reference's 4-byte descriptor width
                         "read_frac": round((8 * F + 8 * n_hit) / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                         # SURVEY.md 8(d)'s own formula with the V2 node width: 8*F + 8*hits + 24*rays
                         "frac_survey": round((8 * F + 8 * n_hit + 24 * n_px) / (kern_ms * 1e-3) / 1e9
                                              / HBM_PEAK_GBS, 5),
                         # the reference's walk from the cube entry (F_ref fetches): the work the kernel
                         # replaces, over its time -- an effective rate, not bytes moved
                         "frac_reference_work": round((bytes_per_launch + 8 * (F_ref - F)) / (kern_ms * 1e-3) / 1e9
                                                      / HBM_PEAK_GBS, 5),
                         "frac_ref_node_width": round((bytes_per_launch - 4 * F) / (kern_ms * 1e-3) / 1e9
                                                      / HBM_PEAK_GBS, 5),
                         "read_frac_ref_node_width": round((4 * F + 8 * n_hit) / (kern_ms * 1e-3) / 1e9
                                                           / HBM_PEAK_GBS, 5),
                         "accountings": "F = the node fetches of the walk the kernel runs (from the beam start, "
                                        "DESIGN.md 3.1d); frac: 8-B V2 node fetches + attachment + hit record + "
                                        "RGBA32F (+ payload) writes; frac_survey: SURVEY 8(d)'s 8*F + 8*hits + 24*rays; "
                                        "frac_reference_work: frac with the reference walk's fetches (F_ref, from the "
                                        "cube entry) in place of F; "
                                        "read_frac: node + attachment reads only (8*F + 8*hits); "
                                        "*_ref_node_width: the same with the reference's 4-byte descriptors (4*F); "
                                        "hbm_frac: what the PMC counters saw cross the fabric",
                         "kernel_source_sha1": digest,
                         "traffic_source": None if pmc is None else pmc.get("source")},
            "cpu_baseline": cpu,
            "c3_plus_shadow_ray": shadow,
        }
        if world > 1:
            out["multi_gpu"] = {
                "frame": f"{W}x{H}", "band_rows": 8, "payload": args.payload,
                "per_pixel_outputs": "every rank: 24-B hit record + 16-B RGBA32F Result of each of its pixels (the "
                                     "N = 1 step's outputs) + its band payload; rank 0 also the display frame's "
                                     "RGBA8 words",
                "preflight": preflight,
                "other_frame": other,
                "per_rank_kernel_gather_assemble_ms": per_rank,
                "render_only_Mrays": round(rays_per_step / (kern_ms_max * 1e-3) / 1e6, 2),
                "gather_ms_rank0": round(stages["gather_ms"], 4), "assemble_ms_rank0": round(stages["assemble_ms"], 4),
                "payload_bytes_per_sending_rank": stages["payload_bytes"],
                "display_rank_deal": deal_info,
                "payload_choice": payload_choice,
                "assembled_frame_check": frame_check,
                "samples_in_flight": samples_n,
                "note": "value overlaps the gather of frame k with the render of frame k+1; render_only_Mrays is "
                        "the frame's rays over the slowest rank's render kernel alone; gather/assemble from a "
                        "serialized pass (events on the gather stream)"}
        if dropin:
            out["dropin_loop"] = dropin
            out["pan"] = pan
        if poses:
            out["extra_poses"] = poses
        if host_path:
            out["host_path"] = host_path
        if in_flight:
            out["frames_in_flight"] = in_flight
        if samples:
            out["samples_in_flight"] = samples
        if split:
            out["strong_split_rehearsal"] = split
        print(json.dumps(out), flush=True)
    rm.close()
    if world > 1:
        dist.destroy_process_group()


def measure_frame(args, rm, W, H, rank, world, dev, stream, dist):
    """One measured frame size: the instrumented fetch count, warmup, K timed steps
    between barrier + synchronize, K more steps with the render kernel bracketed by
    library HIP events, and (N > 1) the serialized stage times and the assembled-frame
    check.  Every rank writes the same per-pixel outputs as the N = 1 step (24-byte hit
    record + RGBA32F Result of each of its pixels) plus, at N > 1, its band payload
    (rank 0: the display frame's RGBA8 words)."""
    import torch
    from raytracingtest_amd import _lib
    sptr = stream.cuda_stream
    gather = deal_info = payload_choice = None
    if world > 1:
        gather, deal_info, payload_choice = choose_payload(args, rm, W, H, rank, world, dev, stream, dist)
        args.payload = gather.payload
        hits = rgba = None
        band = gather.band
        n_px = gather.n_local
    else:
        band = None
        n_px = W * H
        hits = torch.empty(n_px * 24, dtype=torch.uint8, device=dev)
        rgba = None if args.no_rgba else torch.empty(n_px * 4, dtype=torch.float32, device=dev)

    def step():
        if gather is None:
            rm.render_device(W, H, rgba_ptr=None if rgba is None else rgba.data_ptr(), hits_ptr=hits.data_ptr(),
                             stack_mode=args.stack_mode, stream=sptr)
        else:
            gather.step(args.stack_mode)

    def drain():
        if gather is not None:
            gather.drain()

    # instrumented pass (outside the timed region): per-ray fetch counts
    fetch = torch.zeros(max(n_px, 1), dtype=torch.int32, device=dev)
    rm.count_fetches_device(W, H, fetch.data_ptr(), stack_mode=args.stack_mode, band=band, stream=sptr)
    # ... and of the walk the render runs (from the beam start): the node reads the
    # kernel actually makes, the `frac` accounting; the reference's walk above gives frac_reference_work
    fetch_run = torch.zeros_like(fetch)
    rm.set_count_beam(True)
    rm.count_fetches_device(W, H, fetch_run.data_ptr(), stack_mode=args.stack_mode, band=band, stream=sptr)
    rm.set_count_beam(False)
    for _ in range(max(1, args.warmup)):
        step()
    drain()

    # timed region: K steps between barrier + synchronize, right behind the warmup (the host
    # reads of the hit records and fetch counts come after it, so the GPU does not idle between
    # warmup and timing).  HIP events around each step only with SVO_STEP_EVENTS=1
    # (diagnostics): their stream markers add ~8 us to every step they bracket
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    step_events = os.environ.get("SVO_STEP_EVENTS", "0") != "0"
    # one event pair on the launch stream around launches 2..K of the timed region: with one GPU they
    # run back to back, so the span / (K - 1) is the render kernel's mean duration with no per-launch
    # bracket (a bracket around each launch adds ~5 us of marker processing to what it times).  The
    # pair starts at the end of the first launch: the GPU idles from the synchronize until the host's
    # first launch arrives (~140 us under rocprofv3), which would otherwise be spread over the K steps
    span0, span1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    span_n = args.steps - 1 if args.steps > 1 else 1
    if args.steps == 1:
        span0.record(stream)
    for i in range(args.steps):
        if step_events:
            ev[i][0].record(stream)
        step()
        if step_events:
            ev[i][1].record(stream)
        if i == 0 and args.steps > 1:
            span0.record(stream)
    span1.record(stream)
    drain()   # the last frame's assemble (each step assembles the previous frame)
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
    drain()
    kern_ms_events, n_timed = rm.kernel_time()
    rm.set_kernel_timing(False)
    torch.cuda.synchronize(dev)
    if n_timed != args.steps:
        raise RuntimeError(f"kernel timing: {n_timed} launches recorded, {args.steps} expected")
    # the event pair's own cost (the bracketed kernel read longer than the step
    # it belongs to): the same two hipEventRecords around a one-element kernel on the same stream
    floor_ms = event_floor_ms(stream, dev)
    kern_ms_bracket = max(kern_ms_events - floor_ms, 1e-6)
    span_ms = span0.elapsed_time(span1) / span_n
    # N = 1: the timed region's GPU span per launch (only the render kernel runs on the stream at a
    # held view: the beam splat and the order builds happened in the warmup); N > 1: the bracketed
    # kernel (the steps also hold the gather)
    kern_ms = span_ms if gather is None else kern_ms_bracket
    host_hits = (hits if gather is None else gather.local_hits()).cpu().numpy().view(_lib.HIT_DTYPE)
    n_hit = int(np.count_nonzero(host_hits["flags"] & 1))
    F_ref = int(fetch[:n_px].to(torch.int64).sum().item())
    F = int(fetch_run[:n_px].to(torch.int64).sum().item())
    bytes_per_launch = 8 * F + 8 * n_hit + 24 * n_px + (0 if args.no_rgba else 16 * n_px)
    if gather is not None:
        # the RGBA8 display words (rank 0, in the frame) or band payload (3 B RGB / 4 B RGBA8 /
        # 12-B compact records) the kernel also writes
        bytes_per_launch += (4 if rank == 0 else {"rgb8": 3, "rgba8": 4, "compact": 12, "sparse": 3}[args.payload]) * n_px
    stages = gather.stage_times(args.stack_mode, max(3, args.steps // 2)) if gather else None
    frame_check = gather.check_frame(args.stack_mode) if gather is not None and rank == 0 else None
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_max = float(t[0]), float(t[1])
        per_rank = [torch.zeros(3, dtype=torch.float64, device=dev) for _ in range(world)]
        dist.all_gather(per_rank, torch.tensor([kern_ms, stages["gather_ms"], stages["assemble_ms"]],
                                               dtype=torch.float64, device=dev))
        per_rank = [[round(float(v), 4) for v in t.tolist()] for t in per_rank]
    else:
        kern_ms_max = kern_ms
        per_rank = None
    return dict(gather=gather, hits=hits, rgba=rgba, n_px=n_px, n_hit=n_hit, F=F, F_ref=F_ref, host_hits=host_hits,
                band=band,
                deal_info=deal_info, payload_choice=payload_choice, bytes_per_launch=bytes_per_launch,
                elapsed=elapsed, kern_ms=kern_ms, kern_ms_max=kern_ms_max, stages=stages, frame_check=frame_check,
                per_rank=per_rank, step_ms=step_ms, step=step, kern_ms_events=kern_ms_events, floor_ms=floor_ms,
                kern_ms_bracket=kern_ms_bracket, span_ms=span_ms)


def event_floor_ms(stream, dev, n=200):
    """Median time two hipEventRecords on `stream` read around a one-element kernel: what an event
    bracket adds to the kernel it encloses (packet processing before the dispatch and the completion
    signal after it), subtracted from the library's bracketed render-kernel time."""
    import torch
    x = torch.zeros(1, dtype=torch.float32, device=dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    with torch.cuda.stream(stream):
        for _ in range(20):
            x.add_(1.0)
        for a, b in ev:
            a.record(stream)
            x.add_(1.0)
            b.record(stream)
    torch.cuda.synchronize(dev)
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def peer_matrix(devices):
    """hipDeviceCanAccessPeer between every pair of the given device indices."""
    import torch
    return [[None if a == b else bool(torch.cuda.can_device_access_peer(a, b)) for b in devices] for a in devices]


def device_identity(d):
    import torch
    p = torch.cuda.get_device_properties(d)
    return {"index": int(d), "name": p.name,
            "pci": "%04x:%02x:%02x" % (getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", 0),
                                        getattr(p, "pci_device_id", 0))}


def rank_preflight(args, rank, world, dev, dist):
    """N > 1 over torchrun: every rank reports its GPU (index + PCI address); under RCCL
    ("nccl") two ranks on one GPU is a launch error and the run stops here naming them
    (the gloo backend rehearses the N > 1 path with ranks sharing one GPU).  Rank 0
    records the backend, the world size the process group sees and the peer-access
    matrix of the ranks' devices."""
    import torch
    backend = dist.get_backend()
    ident = device_identity(dev.index)
    code = int(ident["pci"].replace(":", ""), 16)
    t = torch.tensor([dev.index, code], dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
    allt = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(allt, t)
    devs = [(int(x[0]), int(x[1])) for x in allt]
    shared = len(set(devs)) < world
    if shared and backend == "nccl":
        dup = {}
        for r, d in enumerate(devs):
            dup.setdefault(d, []).append(r)
        bad = {f"device {d[0]} (pci {d[1]:x})": rs for d, rs in dup.items() if len(rs) > 1}
        raise SystemExit(f"bench.py: ranks share a GPU under RCCL: {bad}; launch one rank per GPU "
                         f"(LOCAL_RANK -> device) or use SVO_BENCH_BACKEND=gloo for a one-GPU rehearsal")
    if rank != 0:
        return None
    used = sorted({d[0] for d in devs})
    return {"backend": backend, "process_group_world_size": dist.get_world_size(), "rank_devices": [d[0] for d in devs],
            "ranks_share_a_gpu": shared, "visible_devices": torch.cuda.device_count(),
            "device_identity_rank0": ident,
            "peer_access_matrix": {"devices": used, "can_access": peer_matrix(used)},
            "rccl_device_tensors": backend == "nccl",
            "note": "under nccl the payload gather and the SVO broadcast move device tensors (RCCL over xGMI); "
                    "under gloo they are staged through host memory (one-GPU rehearsal only)"}


class Gather:
    """One rank's render + gather + assemble pipeline (bench's N > 1 step).

    Every rank renders frame k on its stream R: the display rank (0) straight
    into display frame k (frame layout: its own rows of the RGBA8 frame, and of
    the full hit-record / Result frames for the compact payload), every other
    rank into its band buffers and payload k.  Gather stream G moves the
    payloads to rank 0 in one batch of RCCL sends / receives while R renders
    the next frame; rank 0 then assembles frame k's other rows on R right after
    rendering frame k+1 (svo_assemble_frame, skipping its own part).  Render and
    assemble on one stream cost rank 0 less than the two kernels side by side
    (tools/rank0_cost.py).  Two payload / frame slots."""

    def __init__(self, rm, W, H, rank, world, dev, payload, stream, no_rgba, owner=None):
        import torch
        from raytracingtest_amd import _lib
        from raytracingtest_amd import distributed as D
        self.torch, self._lib, self.D = torch, _lib, D
        self.rm, self.W, self.H, self.rank, self.world, self.dev = rm, W, H, rank, world, dev
        self.payload, self.owner, self.no_rgba, self.R = payload, owner, no_rgba, stream
        self.band = D.rank_band(rank, world, owner=owner)
        self.elem = {"rgb8": 3, "rgba8": 4, "compact": 12, "sparse": 3}[payload]
        rows_max = D.max_band_len(H, world, owner=owner)
        if payload == "sparse":   # head + every pixel a hit + the pack's scratch tail
            part_bytes = _lib.sparse_part_bytes(((W + 7) // 8) * ((rows_max + 7) // 8), rows_max * W)
        else:
            part_bytes = rows_max * W * self.elem
        per = (part_bytes + 3) // 4   # int32 words
        self.G = torch.cuda.Stream(dev)
        self.n_local = D.band_len(H, rank, world, owner=owner) * W
        # the per-step plugin arguments, built once (host time per step matters at N = 8:
        # tools/host_overhead.py)
        self.band_c = _lib.make_band(self.band)
        self.deal_c = _lib.make_band((D.DEFAULT_BAND_ROWS, 0, world) if owner is None
                                     else (D.DEFAULT_BAND_ROWS, 0, world, tuple(owner)))
        if rank == 0:   # display frames, double-buffered
            self.frame8 = [torch.empty(W * H, dtype=torch.int32, device=dev) for _ in range(2)]
            self.fhits = [torch.empty(W * H * 24, dtype=torch.uint8, device=dev) for _ in range(2)]
            self.frgba = [None if no_rgba else torch.empty(W * H * 4, dtype=torch.float32, device=dev)
                          for _ in range(2)]
            # parts[k][0]: the display rank's own (never used) slot of the one-call gather
            self.dummy = torch.empty(per, dtype=torch.int32, device=dev)
            self.parts = [[self.dummy] + [torch.empty(per, dtype=torch.int32, device=dev) for _ in range(1, world)]
                          for _ in range(2)]
            self.parts_c = [(ctypes.c_void_p * world)(None, *[p.data_ptr() for p in self.parts[k][1:]])
                            for k in range(2)]
            self.send = None
        else:
            self.hits = torch.empty(max(self.n_local, 1) * 24, dtype=torch.uint8, device=dev)
            self.rgba = None if no_rgba else torch.empty(max(self.n_local, 1) * 4, dtype=torch.float32, device=dev)
            self.send = [torch.zeros(per, dtype=torch.int32, device=dev) for _ in range(2)]
        self.ev_r = [torch.cuda.Event() for _ in range(2)]   # frame rendered (payload ready)
        self.ev_g = [torch.cuda.Event() for _ in range(2)]   # payloads moved
        self.ev_a = [torch.cuda.Event() for _ in range(2)]   # rank 0: parts of the slot read by its assemble
        self.used = [False, False]
        self.k = 0
        self.pending = None      # rank 0: slot rendered and gathered, not yet assembled
        self.last = None         # slot of the last complete frame
        # bytes one sending rank moves per frame (rank 1's share; rank 0 sends nothing)
        self.payload_bytes = D.band_len(H, 1, world, owner=owner) * W * self.elem

    def release(self):
        """Finish pending work and drop the device buffers (before another frame size)."""
        self.drain()
        self.torch.cuda.synchronize(self.dev)
        for name in ("frame8", "fhits", "frgba", "dummy", "parts", "parts_c", "send", "hits", "rgba", "dense",
                     "cbuf", "cnt_host"):
            if hasattr(self, name):
                setattr(self, name, None)

    def local_hits(self):
        """This rank's hit records (uint8 tensor, band order) of the last render."""
        if self.rank != 0:
            return self.hits[:self.n_local * 24]
        from raytracingtest_amd import band_rows
        rows = self.torch.as_tensor(band_rows(self.H, self.band), device=self.dev)
        return self.fhits[self.last].view(self.H, self.W * 24)[rows].reshape(-1)

    def render(self, k, stack_mode):
        ptr = lambda t: None if t is None else t.data_ptr()
        if self.rank == 0:
            self.rm.render_frame(self.W, self.H, hits=ptr(self.fhits[k]), rgba=ptr(self.frgba[k]),
                                 rgba8=ptr(self.frame8[k]), layout=1, stack_mode=stack_mode, band=self.band_c,
                                 stream=self.R.cuda_stream)
        else:
            if self.used[k]:
                self.R.wait_event(self.ev_g[k])   # payload k sent
            sp = self.send[k].data_ptr()
            self.rm.render_frame(self.W, self.H, hits=ptr(self.hits), rgba=ptr(self.rgba),
                                 rgba8=sp if self.payload == "rgba8" else None,
                                 rgb8=sp if self.payload == "rgb8" else None,
                                 compact=sp if self.payload == "compact" else None,
                                 stack_mode=stack_mode, band=self.band_c, stream=self.R.cuda_stream)
        self.ev_r[k].record(self.R)

    def gather(self, k):
        if self.rank == 0:
            if self.used[k]:
                self.G.wait_event(self.ev_a[k])   # parts k read by the previous assemble
        else:
            self.G.wait_event(self.ev_r[k])
        with self.torch.cuda.stream(self.G):
            self.D.gather_fixed_to_root(self.dummy if self.rank == 0 else self.send[k],
                                        self.parts[k] if self.rank == 0 else None, root=0)
        self.ev_g[k].record(self.G)
        self.used[k] = True

    def assemble(self, k, stream):
        ptrs = self.parts_c[k]
        s = stream.cuda_stream
        if self.payload in ("rgba8", "rgb8", "sparse"):
            fmt = {"rgba8": self._lib.PART_RGBA8, "rgb8": self._lib.PART_RGB8,
                   "sparse": self._lib.PART_SPARSE_RGB8}[self.payload]
            self.rm.assemble_frame(self.W, self.H, ptrs, fmt, rgba8=self.frame8[k].data_ptr(),
                                   skip_part=0, stream=s, deal=self.deal_c)
        else:
            fr = self.frgba[k]
            self.rm.assemble_frame(self.W, self.H, ptrs, self._lib.PART_COMPACT, hits=self.fhits[k].data_ptr(),
                                   rgba=None if fr is None else fr.data_ptr(), rgba8=self.frame8[k].data_ptr(),
                                   skip_part=0, stream=s, deal=self.deal_c)

    def drain(self):
        """Rank 0: assemble the frame still pending (end of a run of steps)."""
        if self.rank == 0 and self.pending is not None:
            k = self.pending
            self.R.wait_event(self.ev_g[k])
            self.assemble(k, self.R)
            self.ev_a[k].record(self.R)
            self.last = k
            self.pending = None

    def step(self, stack_mode):
        k = self.k
        self.k ^= 1
        self.render(k, stack_mode)
        self.gather(k)
        if self.rank == 0:
            self.drain()          # the previous frame's rows from the other ranks, behind this render
            self.pending = k
        else:
            self.last = k

    def stage_times(self, stack_mode, n):
        """Serialized render -> gather -> assemble, events on the gather stream."""
        torch = self.torch
        self.drain()
        g_ms, a_ms = [], []
        for _ in range(n):
            torch.cuda.synchronize(self.dev)
            self.render(0, stack_mode)
            self.R.synchronize()
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(self.G)
            self.gather(0)
            e1.record(self.G)
            if self.rank == 0:
                self.assemble(0, self.G)
                self.ev_a[0].record(self.G)
            e2.record(self.G)
            self.G.synchronize()
            g_ms.append(e0.elapsed_time(e1))
            a_ms.append(e1.elapsed_time(e2))
        self.last, self.k = 0, 1
        return {"gather_ms": float(np.median(g_ms)), "assemble_ms": float(np.median(a_ms)),
                "payload_bytes": self.payload_bytes}

    def check_frame(self, stack_mode):
        """The display frame assembled from the ranks' bands vs the same frame
        rendered whole by the display GPU alone (one launch, no split): RGBA8
        words, and hit records for the compact payload, must be identical."""
        torch = self.torch
        self.drain()
        torch.cuda.synchronize(self.dev)
        k = self.last
        whole8 = torch.empty_like(self.frame8[k])
        whole_hits = torch.empty_like(self.fhits[k]) if self.payload == "compact" else None
        self.rm.render_frame(self.W, self.H, rgba8=whole8.data_ptr(),
                             hits=None if whole_hits is None else whole_hits.data_ptr(),
                             stack_mode=stack_mode, stream=self.R.cuda_stream)
        torch.cuda.synchronize(self.dev)
        bad = int((whole8 != self.frame8[k]).sum().item())
        out = {"pixels": self.W * self.H, "rgba8_mismatches": bad}
        if whole_hits is not None:
            out["hit_record_mismatches"] = int((whole_hits.view(-1, 24) != self.fhits[k].view(-1, 24)).any(1).sum().item())
        return out


class SparseGather(Gather):
    """Gather with the sparse band payload: a sending rank renders
    its dense RGB into a scratch band and the tile hit masks into the head of
    payload k, svo_pack_hits packs the hits' RGB behind the masks, and only
    masks + hits cross xGMI.  The size varies per frame, so the transfer runs one
    step late: step s sends frame s's hit count to rank 0 (4 bytes per rank, on
    the gather stream) and then frame s-1's payload at its exact size, after the
    host has read frame s-1's counts -- by then frame s's render is already
    queued on every GPU, so the host wait does not idle them.  Rank 0 assembles
    frame s-1 behind the render of frame s (misses: sky computed there)."""

    def __init__(self, rm, W, H, rank, world, dev, payload, stream, no_rgba, owner=None):
        super().__init__(rm, W, H, rank, world, dev, payload, stream, no_rgba, owner)
        torch, D = self.torch, self.D
        self.tiles = [((W + 7) // 8) * ((D.band_len(H, m, world, owner=owner) + 7) // 8) for m in range(world)]
        if rank == 0:
            self.cbuf = [torch.zeros(world, dtype=torch.int32, device=dev) for _ in range(2)]
            self.cnt_host = [torch.zeros(world, dtype=torch.int32).pin_memory() for _ in range(2)]
            self.ev_c = [torch.cuda.Event() for _ in range(2)]
        else:
            self.dense = torch.empty(max(self.n_local, 1) * 3, dtype=torch.uint8, device=dev)
            self.cnt_host = [torch.zeros(1, dtype=torch.int32).pin_memory() for _ in range(2)]
        self.sent = 0            # payload bytes of the last frame this rank sent (rank 0: rank 1's)

    def render(self, k, stack_mode):
        if self.rank == 0:
            return super().render(k, stack_mode)
        if self.used[k]:
            self.R.wait_event(self.ev_g[k])   # payload k sent
        s = self.R.cuda_stream
        ptr = lambda t: None if t is None else t.data_ptr()
        nt = self.tiles[self.rank]
        self.rm.render_frame(self.W, self.H, hits=ptr(self.hits), rgba=ptr(self.rgba), rgb8=self.dense.data_ptr(),
                             hitmask=self.send[k].data_ptr(), stack_mode=stack_mode, band=self.band_c, stream=s)
        self.rm.pack_hits(self.W, self.H, self.band_c, self.dense.data_ptr(), self.send[k].data_ptr(), stream=s)
        with self.torch.cuda.stream(self.R):
            self.cnt_host[k].copy_(self.send[k][3 * nt:3 * nt + 1], non_blocking=True)   # the count, byte 12 n
        self.ev_r[k].record(self.R)

    def _part_bytes(self, m, count):
        return self._lib.sparse_head_bytes(self.tiles[m]) + 3 * int(count)

    def gather_counts(self, k):
        """Frame k's hit counts to rank 0 (device to device, then to pinned host)."""
        if self.rank == 0:
            with self.torch.cuda.stream(self.G):
                slots = [self.cbuf[k][m:m + 1] for m in range(self.world)]
                self.D.gather_fixed_to_root(slots[0], slots, root=0)
                self.cnt_host[k].copy_(self.cbuf[k], non_blocking=True)
            self.ev_c[k].record(self.G)
        else:
            nt = self.tiles[self.rank]
            self.G.wait_event(self.ev_r[k])
            with self.torch.cuda.stream(self.G):
                self.D.gather_fixed_to_root(self.send[k][3 * nt:3 * nt + 1], None, root=0)

    def gather(self, k):
        """Frame k's payloads at their exact sizes (its counts gathered a step earlier)."""
        if self.rank == 0:
            self.ev_c[k].synchronize()
            counts = self.cnt_host[k].tolist()
            if self.used[k]:
                self.G.wait_event(self.ev_a[k])   # parts k read by the previous assemble
            parts = [None] + [self.parts[k][m].view(self.torch.uint8)[:self._part_bytes(m, counts[m])]
                              for m in range(1, self.world)]
            with self.torch.cuda.stream(self.G):
                self.D.gather_to_root(None, parts, root=0)
            self.sent = self._part_bytes(1, counts[1])
        else:
            self.ev_r[k].synchronize()
            n = self._part_bytes(self.rank, self.cnt_host[k].item())
            with self.torch.cuda.stream(self.G):
                self.D.gather_to_root(self.send[k].view(self.torch.uint8)[:n], None, root=0)
            self.sent = n
        self.ev_g[k].record(self.G)
        self.used[k] = True

    def drain(self):
        """Send and (rank 0) assemble the frame still pending."""
        if self.pending is None:
            return
        k = self.pending
        self.pending = None
        self.gather(k)
        if self.rank == 0:
            self.R.wait_event(self.ev_g[k])
            self.assemble(k, self.R)
            self.ev_a[k].record(self.R)
        self.last = k

    def step(self, stack_mode):
        k = self.k
        self.k ^= 1
        self.render(k, stack_mode)
        self.gather_counts(k)
        self.drain()             # frame k-1: its payloads, and on rank 0 its assemble behind render k
        self.pending = k

    def stage_times(self, stack_mode, n):
        """Serialized render -> counts -> payload -> assemble, events on the gather stream."""
        torch = self.torch
        self.drain()
        g_ms, a_ms, sent = [], [], []
        for _ in range(n):
            torch.cuda.synchronize(self.dev)
            self.render(0, stack_mode)
            self.R.synchronize()
            e0, e1, e2, e3, e4 = (torch.cuda.Event(enable_timing=True) for _ in range(5))
            e0.record(self.G)
            self.gather_counts(0)
            e1.record(self.G)
            self.G.synchronize()
            e2.record(self.G)
            self.gather(0)
            e3.record(self.G)
            if self.rank == 0:
                self.assemble(0, self.G)
                self.ev_a[0].record(self.G)
            e4.record(self.G)
            self.G.synchronize()
            g_ms.append(e0.elapsed_time(e1) + e2.elapsed_time(e3))
            a_ms.append(e3.elapsed_time(e4))
            sent.append(self.sent)
        self.last, self.k, self.pending = 0, 1, None
        self.payload_bytes = int(np.median(sent))
        return {"gather_ms": float(np.median(g_ms)), "assemble_ms": float(np.median(a_ms)),
                "payload_bytes": self.payload_bytes}


class SamplesGather(Gather):
    """N > 1 samples in flight: every rank traces S jittered samples of its
    bands in ONE launch (svo_render_samples, one wave per sample and tile) and blends them
    into its own band accumulation in _currentSample order (RaytracingMaster.cs:35,70-73,
    AddShader.shader:44-47).  Rank 0 blends straight into the frame-layout accumulation and
    the display frame's words; every other rank into its band accumulation plus the 3-byte
    RGB of the blended band, which moves to rank 0 once per S samples through the Gather
    pipeline (payload k gathered while step k + 1 renders, assembled behind it).  The
    display frame after a step = RGBA8 of the frame accumulated over S more samples.  S is
    a class attribute (samples_gather_class) so weigh_display_rank can rebuild it."""
    S = 4

    def __init__(self, rm, W, H, rank, world, dev, payload, stream, no_rgba, owner=None):
        super().__init__(rm, W, H, rank, world, dev, "rgb8", stream, True, owner)
        from raytracingtest_amd.camera import jitter_offsets
        torch = self.torch
        self.offs = jitter_offsets(4096)
        self.n = 0               # samples blended so far (_currentSample)
        self.count_at = [0, 0]   # samples in display frame k
        self.fhits = self.frgba = self.hits = self.rgba = None   # one-sample outputs, unused here
        px = W * H if rank == 0 else max(self.n_local, 1)
        self.acc = torch.zeros(px * 4, dtype=torch.float32, device=dev)
        torch.cuda.synchronize(dev)

    def local_hits(self):
        raise NotImplementedError("samples in flight write no hit records")

    def render(self, k, stack_mode):
        offs = self.offs[np.arange(self.n, self.n + self.S) % len(self.offs)]
        first = self.n
        self.n += self.S
        self.count_at[k] = self.n
        s = self.R.cuda_stream
        if self.rank == 0:
            self.rm.render_samples(self.W, self.H, offs, first, self.acc.data_ptr(), rgba8=self.frame8[k].data_ptr(),
                                   layout=self._lib.LAYOUT_FRAME, stack_mode=stack_mode, band=self.band_c, stream=s)
        else:
            if self.used[k]:
                self.R.wait_event(self.ev_g[k])   # payload k sent
            self.rm.render_samples(self.W, self.H, offs, first, self.acc.data_ptr(), rgb8=self.send[k].data_ptr(),
                                   stack_mode=stack_mode, band=self.band_c, stream=s)
        self.ev_r[k].record(self.R)

    def check_frame(self, stack_mode):
        """The assembled display frame vs ONE device replaying the same sample sequence
        over the whole frame (one launch per S samples, no split): RGBA8 words identical."""
        torch = self.torch
        self.drain()
        torch.cuda.synchronize(self.dev)
        k = self.last
        n = self.count_at[k]
        acc = torch.zeros(self.W * self.H * 4, dtype=torch.float32, device=self.dev)
        whole8 = torch.empty_like(self.frame8[k])
        torch.cuda.synchronize(self.dev)
        for j in range(0, n, self.S):
            self.rm.render_samples(self.W, self.H, self.offs[np.arange(j, j + self.S) % len(self.offs)], j,
                                   acc.data_ptr(), rgba8=whole8.data_ptr(), stack_mode=stack_mode,
                                   stream=self.R.cuda_stream)
        torch.cuda.synchronize(self.dev)
        return {"pixels": self.W * self.H, "samples_accumulated": n,
                "rgba8_mismatches": int((whole8 != self.frame8[k]).sum().item())}


def samples_gather_class(S):
    return type(f"SamplesGather{S}", (SamplesGather,), {"S": S})


def measure_samples(args, rm, W, H, rank, world, dev, stream, dist, S):
    """The N > 1 samples-in-flight line for one S: weighted deal calibrated as for the
    one-sample line, K pipelined steps between barriers (max over ranks), the render
    kernel's mean (library events, max over ranks) and the assembled-frame check."""
    import torch
    g = samples_gather_class(S)(rm, W, H, rank, world, dev, "rgb8", stream, True)
    g, info = weigh_display_rank(g, args, rm, dist, dev)
    for _ in range(max(1, args.warmup)):
        g.step(args.stack_mode)
    g.drain()
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g.step(args.stack_mode)
    g.drain()
    torch.cuda.synchronize(dev)
    dist.barrier()
    elapsed = time.perf_counter() - t0
    rm.set_kernel_timing(True)
    rm.kernel_time()
    for _ in range(args.steps):
        g.step(args.stack_mode)
    g.drain()
    kern, _ = rm.kernel_time()
    rm.set_kernel_timing(False)
    torch.cuda.synchronize(dev)
    check = g.check_frame(args.stack_mode) if rank == 0 else None
    t = torch.tensor([elapsed, kern], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    per_rank = [torch.zeros(1, dtype=torch.float64, device=dev) for _ in range(world)]
    dist.all_gather(per_rank, torch.tensor([kern], dtype=torch.float64, device=dev))
    g.release()
    ms = float(t[0]) / args.steps * 1e3
    return {"S": S, "ms_per_step": round(ms, 4), "Mrays_per_s": round(S * W * H / (ms * 1e-3) / 1e6, 2),
            "rays_per_step": S * W * H, "kernel_ms_max_rank": round(float(t[1]), 4),
            "per_rank_kernel_ms": [round(float(x[0]), 4) for x in per_rank],
            "display_rank_deal": info, "assembled_frame_check": check}


def choose_payload(args, rm, W, H, rank, world, dev, stream, dist, steps=20):
    """The N > 1 gather of the run: the payload --payload names, or with `auto`
    the faster of rgb8 and sparse.  Each candidate gets its own weighted deal
    (weigh_display_rank) and then runs `steps` pipelined steps between barriers;
    the slowest rank's time decides (all ranks take the same choice).  Sparse
    moves ~0.45x the bytes at a C3 pose but costs every sending rank a pack
    (~11 us) and rank 0 the sky of every miss: it wins when xGMI,
    not the render, bounds the step."""
    import torch
    cands = ["rgb8", "sparse"] if args.payload == "auto" else [args.payload]
    timed = {}
    best = None
    for p in cands:
        cls = SparseGather if p == "sparse" else Gather
        ms = None
        try:
            g = cls(rm, W, H, rank, world, dev, p, stream, args.no_rgba)
            g, info = weigh_display_rank(g, args, rm, dist, dev)
            if len(cands) > 1:
                for _ in range(3):
                    g.step(args.stack_mode)
                g.drain()
                torch.cuda.synchronize(dev)
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(steps):
                    g.step(args.stack_mode)
                g.drain()
                torch.cuda.synchronize(dev)
                t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                ms = float(t[0]) / steps * 1e3
                timed[p] = {"ms_per_step": round(ms, 4), "display_share": info["display_share"]}
        except Exception as e:   # a candidate that fails the same way on every rank is skipped, not fatal
            if len(cands) == 1 or p == cands[0]:
                raise
            print(f"bench.py: payload {p} failed in calibration ({type(e).__name__}: {e}); using {best[1].payload}",
                  file=sys.stderr, flush=True)
            timed[p] = {"error": f"{type(e).__name__}: {e}"[:200]}
            torch.cuda.synchronize(dev)
            continue
        if best is None or (ms is not None and ms < best[0]):
            best = (ms, g, info)
        else:
            del g
    choice = None
    if timed:
        choice = {"mode": "auto", "calibration_steps": steps, "candidates": timed, "chosen": best[1].payload}
    return best[1], best[2], choice


def weigh_display_rank(gather, args, rm, dist, dev):
    """Balance the display rank: it also assembles the frame, so it gets a smaller
    share of the bands (distributed.weighted_owner).  Its share = 1 - (assemble
    time + 3 us frame-layout cost) / render-kernel time, measured here on the
    round-robin deal (max over ranks) unless --display-share fixes it; every rank
    uses rank 0's figure.  Returns the gather to time and a record of the deal."""
    import torch
    share = args.display_share
    measured = None
    if share is None:
        for _ in range(3):
            gather.step(args.stack_mode)
        gather.drain()
        st = gather.stage_times(args.stack_mode, 5)
        rm.set_kernel_timing(True)
        rm.kernel_time()
        for _ in range(5):
            gather.step(args.stack_mode)
        gather.drain()
        kern = rm.kernel_time()[0]
        rm.set_kernel_timing(False)
        t = torch.tensor([kern, st["assemble_ms"] if gather.rank == 0 else 0.0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        kern, asm = float(t[0]), float(t[1])
        share = max(0.0, 1.0 - (asm + 0.003) / kern)
        measured = {"render_kernel_ms_max": round(kern, 4), "display_assemble_ms": round(asm, 4)}
    t = torch.tensor([share], dtype=torch.float64, device=dev)
    dist.broadcast(t, 0)
    share = max(float(t[0]), 1.0 / 8.0)   # at least one band per round: every rank renders
    from raytracingtest_amd import distributed as D
    owner = D.weighted_owner(gather.world, share) or [0] * 8
    info = {"display_share": round(owner.count(0) / 8, 3), "calibration": measured,
            "cycle_bands": len(owner), "rows_rank0": gather.D.band_len(gather.H, 0, gather.world, owner=owner),
            "rows_rank1": gather.D.band_len(gather.H, 1, gather.world, owner=owner)}
    torch.cuda.synchronize(dev)
    if owner.count(0) == 8:   # round-robin
        info["cycle_bands"] = 0
        return type(gather)(gather.rm, gather.W, gather.H, gather.rank, gather.world, dev, gather.payload, gather.R,
                            gather.no_rgba), info
    return type(gather)(gather.rm, gather.W, gather.H, gather.rank, gather.world, dev, gather.payload, gather.R,
                        gather.no_rgba, owner=owner), info


def bench_multidevice(args, svo, cam, W, H, scaling, build_s):
    """One process, N GPUs through the plugin's multi-device context (the Unity
    host's form).  A step renders W x H rays split over the members and leaves the
    N = 1 step's outputs -- 24-B hit records and the RGBA32F Result, plus the
    display RGBA8 words -- for the whole frame on device 0: members send 12-byte
    compact records, from which the display device rebuilds normal and Result."""
    import torch
    from raytracingtest_amd import RaytracingMaster, _lib
    from raytracingtest_amd import distributed as D
    n = args.gpus
    rm = RaytracingMaster(devices=args.device_list, capacity_nodes=len(svo), config=args.svo_config)
    rm.SetSVOBuffer(svo)
    dev0 = torch.device("cuda", args.device_list[0])
    s = torch.cuda.Stream(dev0)
    links = rm.member_links()
    distinct = sorted(set(args.device_list))
    preflight = {"members": [{"device": d, "link": k} for d, k in links],
                 "members_share_a_gpu": len(distinct) < n,
                 "peer_access_matrix": {"devices": distinct, "can_access": peer_matrix(distinct)},
                 "note": "link: how a member's compact payload reaches the display device -- xgmi_peer_pull "
                         "(the assemble kernel reads it over xGMI), peer_copy (hipMemcpyPeerAsync into the display "
                         "device: no peer access), self (same device index: the one-GPU rehearsal)"}

    def sync_all():
        for d in distinct:
            torch.cuda.synchronize(d)

    def measure(Wf, Hf):
        rm.UpdateShaderParameters(cam, Wf, Hf)
        hits = torch.empty(Wf * Hf * 24, dtype=torch.uint8, device=dev0)
        rgba = None if args.no_rgba else torch.empty(Wf * Hf * 4, dtype=torch.float32, device=dev0)
        frame8 = torch.empty(Wf * Hf, dtype=torch.int32, device=dev0)

        def step():
            rm.render_frame(Wf, Hf, hits=hits.data_ptr(), rgba=None if rgba is None else rgba.data_ptr(),
                            rgba8=frame8.data_ptr(), layout=1, stack_mode=args.stack_mode, stream=s.cuda_stream)

        rm.set_band_deal(None)
        for _ in range(max(1, args.warmup)):
            step()
        sync_all()
        # the display device also assembles: the same calibrated weighted deal as the ranks
        share = args.display_share
        if share is None:
            rm.set_kernel_timing(True)
            rm.stage_time(0)
            rm.stage_time(1)
            for _ in range(5):
                step()
            sync_all()
            kern = rm.stage_time(0)[0]       # the slowest member's render kernel
            asm = rm.stage_time(1)[0]
            rm.set_kernel_timing(False)
            share = max(0.0, 1.0 - (asm + 0.003) / kern)
        owner = D.weighted_owner(n, max(share, 1.0 / 8.0))
        deal = None
        if owner is not None and owner.count(0) < 8:
            rm.set_band_deal(owner)
            deal = {"display_share": owner.count(0) / 8, "cycle_bands": len(owner)}
        else:
            owner = None
        for _ in range(max(1, args.warmup)):
            step()
        sync_all()
        t = time.perf_counter()
        for _ in range(args.steps):
            step()
        sync_all()
        elapsed = time.perf_counter() - t
        rm.set_kernel_timing(True)
        rm.stage_time(0)
        rm.stage_time(1)
        for _ in range(args.steps):
            step()
        sync_all()
        kern = [rm.member(i).kernel_time()[0] for i in range(n)]
        asm_ms = rm.stage_time(1)[0]
        rm.set_kernel_timing(False)
        # the display member's algorithmic bytes (its own band: 8 F + 8 hits + 24 + 16 + 4 per pixel)
        band0 = (D.DEFAULT_BAND_ROWS, 0, n) if owner is None else (D.DEFAULT_BAND_ROWS, 0, n, tuple(owner))
        rows0 = D.band_len(Hf, 0, n, owner=owner)
        fetch = torch.zeros(max(rows0 * Wf, 1), dtype=torch.int32, device=dev0)
        m0 = rm.member(0)
        m0.count_fetches_device(Wf, Hf, fetch.data_ptr(), stack_mode=args.stack_mode, band=band0,
                                stream=s.cuda_stream)
        step()
        sync_all()
        F = int(fetch.to(torch.int64).sum().item())
        from raytracingtest_amd import band_rows
        ys = torch.as_tensor(band_rows(Hf, band0), device=dev0)
        h0 = hits.view(Hf, Wf * 24)[ys].reshape(-1).cpu().numpy().view(_lib.HIT_DTYPE)
        n_hit0 = int(np.count_nonzero(h0["flags"] & 1))
        bytes0 = 8 * F + 8 * n_hit0 + (24 + (0 if args.no_rgba else 16) + 4) * rows0 * Wf
        # the assembled frame vs the same frame rendered whole by a separate one-device
        # context on the display device (one launch, no split): every output
        one = RaytracingMaster(device=dev0.index, capacity_nodes=len(svo))
        one.SetSVOBuffer(svo)
        one.UpdateShaderParameters(cam, Wf, Hf)
        w_hits, w8 = torch.empty_like(hits), torch.empty_like(frame8)
        w_rgba = None if rgba is None else torch.empty_like(rgba)
        one.render_frame(Wf, Hf, hits=w_hits.data_ptr(), rgba=None if w_rgba is None else w_rgba.data_ptr(),
                         rgba8=w8.data_ptr(), layout=1, stack_mode=args.stack_mode, stream=s.cuda_stream)
        torch.cuda.synchronize(dev0)
        check = {"pixels": Wf * Hf, "rgba8_mismatches": int((w8 != frame8).sum().item()),
                 "hit_record_mismatches": int((w_hits.view(-1, 24) != hits.view(-1, 24)).any(1).sum().item()),
                 "rgba32f_mismatches": None if rgba is None else
                 int((w_rgba.view(-1, 4) != rgba.view(-1, 4)).any(1).sum().item())}
        one.close()
        ms = elapsed / args.steps * 1e3
        return {"ms": ms, "kern": kern, "asm_ms": asm_ms, "deal": deal, "check": check, "bytes0": bytes0,
                "F0": F, "rows0": rows0}

    def measure_samples_md(S):
        """Samples in flight through the multi-device context (svo_render_samples): every
        member blends S samples of its bands on its own device, the display device
        assembles the blended frame's words; checked against one device replaying the
        same sample sequence over the whole frame."""
        from raytracingtest_amd.camera import jitter_offsets
        rm.UpdateShaderParameters(cam, W, H)
        rm.set_band_deal(None)
        offs = jitter_offsets(4096)
        acc = torch.zeros(W * H * 4, dtype=torch.float32, device=dev0)
        frame8 = torch.zeros(W * H, dtype=torch.int32, device=dev0)
        sync_all()
        cnt = [0]

        def step():
            j = cnt[0]
            rm.render_samples(W, H, offs[np.arange(j, j + S) % len(offs)], j, acc.data_ptr(), rgba8=frame8.data_ptr(),
                              layout=_lib.LAYOUT_FRAME, stack_mode=args.stack_mode, stream=s.cuda_stream)
            cnt[0] += S

        for _ in range(max(1, args.warmup)):
            step()
        sync_all()
        t = time.perf_counter()
        for _ in range(args.steps):
            step()
        sync_all()
        ms = (time.perf_counter() - t) / args.steps * 1e3
        one = RaytracingMaster(device=dev0.index, capacity_nodes=len(svo))
        one.SetSVOBuffer(svo)
        one.UpdateShaderParameters(cam, W, H)
        acc1 = torch.zeros_like(acc)
        w8 = torch.zeros_like(frame8)
        torch.cuda.synchronize(dev0)
        for j in range(0, cnt[0], S):
            one.render_samples(W, H, offs[np.arange(j, j + S) % len(offs)], j, acc1.data_ptr(), rgba8=w8.data_ptr(),
                               stack_mode=args.stack_mode, stream=s.cuda_stream)
        torch.cuda.synchronize(dev0)
        bad = int((w8 != frame8).sum().item())
        one.close()
        return {"S": S, "ms_per_step": round(ms, 4), "Mrays_per_s": round(S * W * H / (ms * 1e-3) / 1e6, 2),
                "assembled_frame_check": {"pixels": W * H, "samples_accumulated": cnt[0], "rgba8_mismatches": bad}}

    r = measure(W, H)
    samples_md = None
    if args.extras:
        samples_md = {"frame": f"{W}x{H}", "per_samples": [measure_samples_md(S) for S in (1, 2, 4, 8)],
                      "note": "S jittered samples of the frame per step through the multi-device context "
                              "(svo_render_samples), rays = S x W x H per step; value is one sample per step"}
    other = None
    if args.extras and args.cfg_gpus == 1:
        other_scaling = "weak" if scaling == "strong" else "strong"
        Wo, Ho = D.weak_frame(args.width, args.height, n) if other_scaling == "weak" else (args.width, args.height)
        ro = measure(Wo, Ho)
        other = {"scaling": other_scaling, "frame": f"{Wo}x{Ho}", "rays_per_step": Wo * Ho,
                 "value": round(Wo * Ho / (ro["ms"] * 1e-3) / 1e6, 2), "unit": "Mrays/s",
                 "ms_per_step": round(ro["ms"], 4), "per_device_kernel_ms": [round(k, 4) for k in ro["kern"]],
                 "assemble_ms": round(ro["asm_ms"], 4), "assembled_frame_check": ro["check"]}
    rm.close()
    ms = r["ms"]
    achieved = r["bytes0"] / (r["kern"][0] * 1e-3) / 1e9
    kind = "Menger" if args.svo == "menger" else "Custom1"
    print(json.dumps({
        "metric": METRIC, "value": round(W * H / (ms * 1e-3) / 1e6, 2), "unit": "Mrays/s", "n_gpus": n,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "f32",
        "data": ("synthetic: 256^3 Menger sponge surface SVO (SURVEY.md 8(d) C2)" if args.svo == "menger" else
                 "synthetic: Custom1 OpenSimplex(seed 7) terrain SVO built on-GPU by the NaiveCreator restatement"),
        "config": {"workload": (f"{args.config} depth-{args.max_level - 1} ({1 << (args.max_level - 1)}^3) {kind} SVO, "
                                f"{W}x{H} primary rays, {args.camera} camera"),
                   "parallelism": f"multidevice{n}x8rows+xgmi_pull(compact)", "build_s": round(build_s, 2),
                   "svo_nodes": len(svo), "stack_mode": "hlsl" if args.stack_mode == 0 else "exact"},
        "roofline": {"bound": "latency", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "kernel": "render_tile_kernel on the display device (its own bands), library HIP events",
                     "kernel_ms": round(r["kern"][0], 4), "kernel_ms_max_member": round(max(r["kern"]), 4),
                     "algorithmic_bytes_per_launch": r["bytes0"],
                     "bytes_formula": "display device's rays: 8*F + 8*hits + 24 (hit record) + 16 (RGBA32F) + 4 (RGBA8)"},
        "multi_gpu": {"devices": args.device_list, "preflight": preflight,
                      "per_pixel_outputs": "hit records + RGBA32F Result + RGBA8 of the whole frame on device 0 "
                                           "(the N = 1 step's outputs + display words); members send 12-B compact "
                                           "records",
                      "per_device_kernel_ms": [round(k, 4) for k in r["kern"]],
                      "assemble_ms": round(r["asm_ms"], 4), "display_device_deal": r["deal"],
                      "assembled_frame_check": r["check"], "other_frame": other,
                      "samples_in_flight": samples_md},
    }), flush=True)


def frames_in_flight(rm, W, H, args, dev, n_streams=3):
    """Throughput with consecutive frames on rotating streams (own output
    buffers each; the plugin keeps per-stream dispatch-order state, so their
    renders overlap and the next frame's waves fill one frame's ramp-down;
    3 streams: 2 sometimes share a hardware queue, tools/overlap_experiment.py).
    Reported beside `value`, which -- like the roofline's kernel time -- is
    measured with one frame at a time."""
    import torch
    streams = [torch.cuda.Stream(dev) for _ in range(n_streams)]
    outs = [(torch.empty(W * H * 24, dtype=torch.uint8, device=dev),
             None if args.no_rgba else torch.empty(W * H * 4, dtype=torch.float32, device=dev))
            for _ in range(n_streams)]

    def step(i):
        h, c = outs[i % n_streams]
        rm.render_device(W, H, rgba_ptr=None if c is None else c.data_ptr(), hits_ptr=h.data_ptr(),
                         stack_mode=args.stack_mode, stream=streams[i % n_streams].cuda_stream)

    for i in range(2 * n_streams + 4):
        step(i)
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t) / args.steps * 1e3
    return {"streams": n_streams, "ms_per_frame": round(ms, 4), "Mrays_per_s": round(W * H / (ms * 1e-3) / 1e6, 2)}


def samples_in_flight(rm, W, H, args, dev, stream, sizes=(1, 2, 4, 8), floor_ms=0.0):
    """Samples in flight on one GPU (svo_render_samples): a step traces S jittered samples
    of the frame in ONE launch (one wave per sample and 8x8 tile, cost-ordered) and blends
    them into the accumulation in _currentSample order (RaytracingMaster.cs:35,70-73,
    AddShader.shader:44-47).  Rate = S x W x H rays per step.  Reported beside `value`
    (one sample per step, the metric); the N > 1 form is multi_gpu.samples_in_flight."""
    import torch
    from raytracingtest_amd.camera import jitter_offsets
    offs = jitter_offsets(4096)
    acc = torch.zeros(W * H * 4, dtype=torch.float32, device=dev)
    frame8 = torch.empty(W * H, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    out = {}
    n = 0
    for S in sizes:
        def step():
            nonlocal n
            rm.render_samples(W, H, offs[np.arange(n, n + S) % len(offs)], n,
                              acc.data_ptr(), rgba8=frame8.data_ptr(), stack_mode=args.stack_mode,
                              stream=stream.cuda_stream)
            n += S
        for _ in range(3):
            step()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t) / args.steps * 1e3
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.steps):   # the GPU span per launch, as the render kernel's kernel_ms
            step()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        kern = e0.elapsed_time(e1) / args.steps
        out[str(S)] = {"ms_per_step": round(ms, 4), "kernel_ms": round(kern, 4),
                       "Mrays_per_s": round(S * W * H / (ms * 1e-3) / 1e6, 2),
                       "kernel_Mrays_per_s": round(S * W * H / (kern * 1e-3) / 1e6, 2)}
    return {"per_samples": out, "outputs": "RGBA32F accumulation (read + written) + display RGBA8 of the blended frame",
            "note": "S jittered samples per launch, rays = S x W x H per step; primary rays only"}


def strong_split_bands(rm, W, H, args, dev, stream, hits, rgba, kern_ms, floor_ms, counts=(2, 4, 8), timed=150):
    """One-GPU rehearsal of the metric's frame split over N GPUs: every rank's
    round-robin 8-row band of the same frame rendered alone on this GPU (the launch each GPU of an
    N-way split runs, segmented heavy tiles and loop form chosen by the library as there), its
    GPU time per launch (one event pair around `timed` back-to-back launches after a warmup, as the
    one-GPU kernel_ms), and the predicted N-GPU speed-up of the one-sample frame = this run's kernel_ms over
    the slowest rank's band.  The RCCL gather and display-rank assemble are not in it (they
    overlap the next frame's render)."""
    import torch
    out = {}
    for N in counts:
        per = []
        for r in range(N):
            band = (8, r, N)
            for _ in range(30):
                rm.render_frame(W, H, hits=hits.data_ptr(), rgba=None if rgba is None else rgba.data_ptr(),
                                stack_mode=args.stack_mode, band=band, stream=stream.cuda_stream)
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(timed):
                rm.render_frame(W, H, hits=hits.data_ptr(), rgba=None if rgba is None else rgba.data_ptr(),
                                stack_mode=args.stack_mode, band=band, stream=stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            per.append(e0.elapsed_time(e1) / timed)
        torch.cuda.synchronize(dev)
        out[str(N)] = {"band_kernel_ms_per_rank": [round(x, 4) for x in per], "slowest_rank_ms": round(max(per), 4),
                       "predicted_speedup": round(kern_ms / max(per), 3)}
    return {"per_gpus": out, "frame": f"{W}x{H}", "one_gpu_kernel_ms": round(kern_ms, 4),
            "note": "each rank's round-robin 8-row band rendered alone on ONE GPU (hit records + RGBA32F), "
                    "render kernel only; predicted_speedup = one_gpu_kernel_ms / slowest_rank_ms, gather excluded"}


def host_path_rates(rm, W, H, args, n=5):
    """PCIe-inclusive frame times of the drop-in's blocking host entry points (never
    `value`): svo_render (RGBA32F Result + 24-B hit records to the host, 40 B/px)
    and svo_render_progressive (sample rendered and accumulated on the GPU, the
    display RGBA8 frame to the host, 4 B/px) -- what the Unity host pays per frame."""
    out = {}
    reuse = rm.Render(W, H, stack_mode=args.stack_mode)   # a render loop's arrays, written again every frame
    for name, fn, k in (("svo_render_rgba32f_hits", lambda: rm.Render(W, H, stack_mode=args.stack_mode, out=reuse), 10),
                        ("svo_render_rgba32f_hits_fresh_arrays", lambda: rm.Render(W, H, stack_mode=args.stack_mode), n),
                        ("svo_render_progressive_rgba8", lambda: rm.RenderProgressive(W, H, stack_mode=args.stack_mode),
                         n),
                        # the pipelined entry point: a pointer to the previous frame in pinned memory
                        # (copy=False: what LoadRawTextureData receives), D2H overlapping the next render
                        ("svo_render_progressive_async_rgba8",
                         lambda: rm.RenderProgressiveAsync(W, H, stack_mode=args.stack_mode, copy=False), 50),
                        ("svo_render_progressive_async_rgb24",
                         lambda: rm.RenderProgressiveAsync(W, H, stack_mode=args.stack_mode, copy=False, rgb=True), 50)):
        fn()
        fn()
        t = time.perf_counter()
        for _ in range(k):
            fn()
        ms = (time.perf_counter() - t) / k * 1e3
        bpp = 40 if name.startswith("svo_render_rgba") else 3 if name.endswith("rgb24") else 4
        out[name] = {"ms_per_frame": round(ms, 3), "Mrays_per_s": round(W * H / (ms * 1e-3) / 1e6, 1),
                     "host_bytes_per_frame": W * H * bpp, "frames": k}
    for name in ("svo_render_progressive_async_rgba8", "svo_render_progressive_async_rgb24"):
        out[name]["note"] = ("each call returns the previous frame's pinned pixels (D2H overlapping the next "
                             "render); the caller's own copy of them is not included")
    return out


def dropin_loop_rates(rm, W, H, args, dev, stream, frames=300):
    """The drop-in's own frame loop, measured beside `value` (which repeats one
    frame at pixel offset (0.5, 0.5)).  RaytracingMaster.OnRenderImage draws a fresh
    _PixelOffset = (Random.value, Random.value) every frame (RaytracingMaster.cs:35), blends the
    sample in with _Sample = _currentSample (:70-73) and restarts the blend whenever the camera moves
    (:44-47); the C# shim does the same through svo_render_progressive_async (RGB24).  Three loops:
      fixed   -- held view, offset (0.5, 0.5) every frame (value's ray set);
      jitter  -- held view, a new seeded offset every frame (the `dropin_loop` key);
      pan     -- a new view AND a new offset every frame, _currentSample 0 each time (the `pan` key;
                 camera.pan_cameras: the pose's eye circling by 2 mrad per frame).
    Each loop is timed twice: (1) the plugin's pipelined progressive entry point on the host clock
    (render + AddShader blend + RGB24 pack + D2H of the previous frame into pinned memory, the call
    the shim makes per frame) and, with the library's per-launch events, its render kernel; (2) the
    render alone through svo_render_device on the bench stream with value's outputs (hit record +
    RGBA32F), its GPU span per frame over launches 2..K exactly as value's kernel_ms (the beam splat of
    a new view runs on that stream and is in the pan's span; the order builds run beside it)."""
    import torch
    from raytracingtest_amd import _lib
    from raytracingtest_amd.camera import column_major, jitter_offsets, main_light, pan_cameras
    L = _lib.lib()
    offs = jitter_offsets(frames + 64)
    light = np.ascontiguousarray(main_light(), np.float32)
    cams = pan_cameras(args.camera, frames + 64)
    views = []
    for c in cams:
        c2w, ip = c.uniforms(W, H)
        views.append((column_major(c2w), column_major(ip)))
    ptrs = [(c.ctypes.data, p.ctypes.data) for c, p in views]   # (the arrays stay alive in `views`)
    lptr = light.ctypes.data
    offl = [(float(x), float(y)) for x, y in offs]
    hits = torch.empty(W * H * 24, dtype=torch.uint8, device=dev)
    rgba = torch.empty(W * H * 4, dtype=torch.float32, device=dev)
    sptr = stream.cuda_stream
    hptr, rptr = hits.data_ptr(), rgba.data_ptr()
    ctx = rm._ctx

    def set_cam(kind, k):   # the host's per-frame work kept small: the GPU, not Python, is measured
        c, p = ptrs[k if kind == "pan" else 0]
        ox, oy = (0.5, 0.5) if kind == "fixed" else offl[k]
        if L.svo_set_camera(ctx, c, p, ox, oy, lptr) != 0:
            _lib.check(-1, "svo_set_camera")

    ptr = ctypes.c_void_p()
    state = {"sample": 0}

    def progressive(kind, k):
        set_cam(kind, k)
        s = 0 if kind == "pan" else state["sample"]
        _lib.check(L.svo_render_progressive_async(rm._ctx, W, H, args.stack_mode, s, _lib.PIXELS_RGB8,
                                                  ctypes.byref(ptr)), "svo_render_progressive_async")
        state["sample"] = s + 1

    def device(kind, k):
        set_cam(kind, k)
        if L.svo_render_device(ctx, W, H, args.stack_mode, None, rptr, hptr, sptr) != 0:
            _lib.check(-1, "svo_render_device")

    out = {}
    for kind in ("fixed", "jitter", "pan"):
        state["sample"] = 0
        r = {}
        # (1) the pipelined drop-in call, host clock; then its render kernel by the library's events
        for k in range(30):
            progressive(kind, k)
        _lib.check(L.svo_progressive_last(rm._ctx, ctypes.byref(ptr)), "svo_progressive_last")
        t = time.perf_counter()
        for k in range(frames):
            progressive(kind, k)
        _lib.check(L.svo_progressive_last(rm._ctx, ctypes.byref(ptr)), "svo_progressive_last")
        ms = (time.perf_counter() - t) / frames * 1e3
        rm.set_kernel_timing(True)
        rm.kernel_time()
        for k in range(frames):
            progressive(kind, k)
        kev, n = rm.kernel_time()
        rm.set_kernel_timing(False)
        _lib.check(L.svo_progressive_last(rm._ctx, ctypes.byref(ptr)), "svo_progressive_last")
        r["progressive_async_rgb24"] = {"ms_per_frame": round(ms, 4), "Mrays_per_s": round(W * H / (ms * 1e-3) / 1e6, 1),
                                        "kernel_ms_events": round(kev, 4)}
        # (2) the render alone, value's method
        for k in range(30):
            device(kind, k)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for k in range(frames):
            device(kind, k)
            if k == 0:
                e0.record(stream)
        t_issue = time.perf_counter() - t
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t) / frames * 1e3
        span = e0.elapsed_time(e1) / (frames - 1)
        r["render_device"] = {"ms_per_frame": round(ms, 4), "kernel_ms": round(span, 4),
                              "host_issue_ms_per_frame": round(t_issue / frames * 1e3, 4),
                              "Mrays_per_s": round(W * H / (span * 1e-3) / 1e6, 1)}
        out[kind] = r
    # leave the context at the bench pose, offset (0.5, 0.5)
    set_cam("fixed", 0)
    f, j, p = out["fixed"], out["jitter"], out["pan"]
    ratio = lambda a, b: round(a / b, 4)   # noqa: E731
    dropin = {"frames": frames, "fixed_offset": f, "jittered": j,
              "kernel_vs_fixed_offset": ratio(j["render_device"]["kernel_ms"], f["render_device"]["kernel_ms"]),
              "kernel_events_vs_fixed_offset": ratio(j["progressive_async_rgb24"]["kernel_ms_events"],
                                                     f["progressive_async_rgb24"]["kernel_ms_events"]),
              "Mrays_per_s": j["render_device"]["Mrays_per_s"],
              "note": "svo_render_progressive_async RGB24 (the C# shim's per-frame call) with a new seeded "
                      "_PixelOffset per frame at a held view; kernel_ms = render_device span per frame under the "
                      "same jitter (value's method); fixed_offset = the same loops at (0.5, 0.5)"}
    pan = {"frames": frames, "moving": p,
           "frame_vs_held": ratio(p["render_device"]["ms_per_frame"], j["render_device"]["ms_per_frame"]),
           "kernel_vs_held": ratio(p["render_device"]["kernel_ms"], j["render_device"]["kernel_ms"]),
           "progressive_frame_vs_held": ratio(p["progressive_async_rgb24"]["ms_per_frame"],
                                              j["progressive_async_rgb24"]["ms_per_frame"]),
           "Mrays_per_s": p["render_device"]["Mrays_per_s"],
           "note": "the same loops with a new view every frame (eye circling the pose by 2 mrad per frame, "
                   "camera.pan_cameras) and _currentSample reset each frame; *_vs_held against the jittered "
                   "held view (dropin_loop)"}
    return dropin, pan


def extra_poses(rm, args, W, H, hits, rgba, sptr, dev):
    """Kernel time and ray rate of the same frame from the other camera poses
    (overview and the Main.unity pose; plus a terrain-facing one)."""
    import torch
    from raytracingtest_amd.camera import CAMERAS
    out = {}
    for name in ("overview", "main", "terrain", "flyover"):
        if name == args.camera:
            continue
        rm.UpdateShaderParameters(CAMERAS[name](), W, H)
        for _ in range(10):
            rm.render_device(W, H, rgba_ptr=None if rgba is None else rgba.data_ptr(), hits_ptr=hits.data_ptr(),
                             stack_mode=args.stack_mode, stream=sptr)
        rm.set_kernel_timing(True)
        rm.kernel_time()
        for _ in range(20):
            rm.render_device(W, H, rgba_ptr=None if rgba is None else rgba.data_ptr(), hits_ptr=hits.data_ptr(),
                             stack_mode=args.stack_mode, stream=sptr)
        ms, _ = rm.kernel_time()
        rm.set_kernel_timing(False)
        torch.cuda.synchronize(dev)
        h = hits.cpu().numpy().view(np.dtype([("parent", "<u4"), ("m", "<u4"), ("r", "<u4", 4)]))
        hit_frac = float(np.count_nonzero((h["m"] >> 16) & 1)) / (W * H)
        out[name] = {"kernel_ms": round(ms, 4), "Mrays_per_s_kernel": round(W * H / (ms * 1e-3) / 1e6, 1),
                     "hit_fraction": round(hit_frac, 4)}
    rm.UpdateShaderParameters(CAMERAS[args.camera](), W, H)
    return out


def pmc_traffic(workload, digest):
    """The committed rocprofv3 PMC summary (profiles/pmc_summary.json,
    tools/pmc_summary.py) when it was taken on this workload AND this kernel
    build (source digest), else None."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    if d.get("workload") != workload or d.get("kernel_source_sha1") != digest:
        return None
    return d


def cpu_baseline(args, svo, cam, gpu_hits):
    """Oracle ("port") on every CPU this job may use, over rows of the same
    frame, bounded by --cpu-seconds; the rows it traces are also compared with
    the GPU records.  Plus a 1-thread figure."""
    from oracle import oracle as orc
    from raytracingtest_amd.camera import main_light

    W, H = args.width, args.height
    info = host_cpu_info()
    threads = info["usable_cpus"]
    c2w, inv_proj = cam.uniforms(W, H)
    ocam = orc.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
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
                      f"{threads} threads (every CPU this job may use: affinity {info['affinity_cpus']}, cgroup quota "
                      f"{info['cgroup_cpu_quota']}), {secs:.1f} s; 1-thread rate on 8 rows: {one_core:.3f} Mrays/s",
            "one_core_mrays": round(one_core, 4), "host": info,
            "parity_rays_checked": int(len(pix)), "parity_rays_mismatched": mism}


if __name__ == "__main__":
    main()
