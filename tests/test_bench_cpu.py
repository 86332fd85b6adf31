"""bench.py contract on CPU: ``--gpus 2`` run bare (no RANK/WORLD_SIZE) starts
torch.distributed.run itself as a child, two gloo ranks join, and exactly one
JSON line comes back with the world size and the collectives that ran."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def test_bench_self_launches_two_ranks(tmp_path):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--kernels", "torch",
                        "--arch", "resnet18", "--batch-size", "2", "--image-size", "32", "--steps", "2",
                        "--warmup", "1"], cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["world_size"] == 2 and out["config"]["comm_nranks"] == 2
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 4
    assert out["config"]["collectives_per_step"] >= 1
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["dtype"] == "fp32"  # the CPU torch path does not autocast: say so
    ov = out["config"]["comm_overlap"]  # bucket timeline of a step after the timed region (parallel/ddp.py)
    nb = len(out["config"]["bucket_plan_mb"])
    assert ov["issue_order"] == list(range(nb)) and len(ov["bucket_issue_ms"]) == nb
    assert ov["exposed_comm_ms"] >= 0 and ov["backward_ms"] > 0
