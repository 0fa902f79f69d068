"""bench.py under torch.distributed.run at world size 1: the data-parallel path
(process group on backend "nccl" = RCCL, the gather of the packed detections to
rank 0 on device tensors) runs on the GPU, and rank 0's gathered rows equal its
own NMS results (bench.py records the check). Marked gpu.

The N > 1 gather logic itself is covered on CPU by tests/test_dist_gloo.py.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("extra", [[], ["--serial"]])
def test_bench_under_torchrun_world1_gathers_over_rccl(gpu, extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--no-roofline", *extra]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([line for line in r.stdout.splitlines() if line.startswith("{")][-1])
    assert rec["n_gpus"] == 1 and rec["value"] > 0
    assert rec["gather"] is not None and "1 rank(s)" in rec["gather"], rec["gather"]
    assert rec["gather"].endswith("match: True"), rec["gather"]
