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
    env = dict(os.environ, SVO_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "6", "--warmup", "2", "--payload", payload, "--cpu-seconds", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 6 and d["scaling"] == "weak" and d["value"] > 0
    mg = d["multi_gpu"]
    assert mg["assembled_frame_check"]["rgba8_mismatches"] == 0
    if payload == "compact":
        assert mg["assembled_frame_check"]["hit_record_mismatches"] == 0
    if payload == "auto":
        assert mg["payload"] in ("rgb8", "sparse")
        assert set(mg["payload_choice"]["candidates"]) == {"rgb8", "sparse"}
    else:
        assert mg["payload"] == payload
    assert d["config"]["parallelism"].endswith(f"rccl_gather({mg['payload']})")
