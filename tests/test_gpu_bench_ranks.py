"""bench.py's N > 1 path end to end on one GPU (the driver's SCALE run uses the
same code over RCCL, one GPU per rank): two torchrun ranks share cuda:0 over
gloo (SVO_BENCH_BACKEND=gloo, host-staged gathers), render their bands, move
their payloads to rank 0 (dense RGB, compact records, or the sparse hit payload
with its per-frame count exchange, and `auto`, which calibrates rgb8 against
sparse), and rank 0 compares its assembled frame with a one-launch render of
the whole frame.  The rates of ranks time-slicing one GPU mean nothing; the
frame check and the JSON contract are what is asserted.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("payload", ["auto", "sparse", "compact"])
def test_two_ranks_assemble_the_whole_frame(gpu, payload):
    """`value` is the metric's 1920x1080 frame split over the ranks (strong); with
    the extras on (payload auto) the weak frame is measured beside it, labelled,
    with its own assembled-frame check.  Rank 0 records the preflight."""
    env = dict(os.environ, SVO_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    extras = [] if payload == "auto" else ["--no-extras"]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "6", "--warmup", "2", "--payload", payload, "--cpu-seconds", "0"] + extras
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 6 and d["scaling"] == "strong" and d["value"] > 0
    assert "1920x1080 primary rays" in d["config"]["workload"] and d["config"]["rays_per_step"] == 1920 * 1080
    assert d["roofline"]["achieved"] > 0 and d["roofline"]["algorithmic_bytes_per_launch"] > 0
    mg = d["multi_gpu"]
    assert mg["frame"] == "1920x1080"
    assert mg["assembled_frame_check"]["rgba8_mismatches"] == 0
    pf = mg["preflight"]
    assert pf["backend"] == "gloo" and pf["process_group_world_size"] == 2 and pf["ranks_share_a_gpu"]
    if payload == "compact":
        assert mg["assembled_frame_check"]["hit_record_mismatches"] == 0
    if payload == "auto":
        assert mg["payload"] in ("rgb8", "sparse")
        assert set(mg["payload_choice"]["candidates"]) == {"rgb8", "sparse"}
        o = mg["other_frame"]
        assert o["scaling"] == "weak" and o["frame"] != "1920x1080" and o["value"] > 0
        assert o["assembled_frame_check"]["rgba8_mismatches"] == 0
        # samples in flight across the ranks: S jittered samples per launch and rank, the
        # assembled accumulation equal to one device replaying the same samples
        sif = mg["samples_in_flight"]["per_samples"]
        assert [e["S"] for e in sif] == [1, 2, 4, 8]
        for e in sif:
            assert e["rays_per_step"] == e["S"] * 1920 * 1080 and e["Mrays_per_s"] > 0
            assert e["assembled_frame_check"]["rgba8_mismatches"] == 0, e
    else:
        assert mg["payload"] == payload and mg["other_frame"] is None
    assert d["config"]["parallelism"].endswith(f"rccl_gather({mg['payload']})")


@pytest.mark.parametrize("copy", [False, True])
def test_multidevice_bench_like_for_like(gpu, copy):
    """bench.py --gpus 2 without torchrun (the multi-device context, both members on
    cuda:0): the step leaves hit records + RGBA32F + RGBA8 of the whole frame on the
    display device, every output equal to a one-launch render; svo_config.peer_copy 1 takes
    the copy fallback a member without peer access gets (svo_create_multi)."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--devices", "0,0", "--steps", "6", "--warmup", "2",
           "--cpu-seconds", "0", "--no-extras", "--set", f"peer_copy={1 if copy else 0}"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["scaling"] == "strong" and d["roofline"]["achieved"] > 0
    mg = d["multi_gpu"]
    assert [m["link"] for m in mg["preflight"]["members"]] == ["self", "peer_copy" if copy else "self"]
    chk = mg["assembled_frame_check"]
    assert chk["rgba8_mismatches"] == 0 and chk["hit_record_mismatches"] == 0 and chk["rgba32f_mismatches"] == 0
