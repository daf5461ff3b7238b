"""The RCCL branches of the multi-GPU path on a real communicator (world size 1, one GPU).

The N > 1 rehearsals on one GPU run over gloo, which stages device tensors through host
memory; the branches that hand device tensors to RCCL (broadcast_svo, the payload gathers,
accumulate_samples, bench.rank_preflight) run for real only here -- in a child process, so
the communicator never lives in the test runner.  tools/rccl_world1.py lists the checks."""
import json
import os
import socket
import subprocess
import sys

import pytest

from tests.conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
def test_rccl_branches_world1():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_world1.py")], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["backend"] == "nccl" and out["world"] == 1
    assert out["broadcast_svo"] == out["gathers"] == out["all_reduce"] == "ok"
    assert out["render_from_broadcast_pool"] == "identical"
