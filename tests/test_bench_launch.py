"""bench.py --gpus N self-launch: started without a launcher, the bench
spawns N ranks under torch.distributed.run itself (reference: env-driven ranks under a launcher,
main.py:338-344, main.sh:1-2). --dry-run replaces the HIP step by a gloo gather on the CPU, so the
launcher, the rank layout, the max-over-ranks timing and the single JSON line are checked here."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "3",
                        "--warmup", "1", "--batch", "4", *extra],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return lines, p


def test_gpus2_self_launches_two_ranks():
    lines, p = _run("--gpus", "2")
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["ranks_gathered"] == [0, 1]          # both ranks ran and reached the collective
    assert rec["config"]["global_batch"] == 8 and rec["config"]["parallelism"] == "dp2"
    assert "launching 2 ranks" in p.stderr


def test_gpus1_runs_in_process():
    lines, p = _run("--gpus", "1")
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 1 and rec["ranks_gathered"] == [0]
    assert "launching" not in p.stderr
