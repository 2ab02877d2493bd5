"""The multi-rank launcher the driver's scaling run uses: `python bench.py --gpus N`.

bench.py started with --gpus 2 and no torch.distributed environment starts its own two ranks with
torch.distributed.run (a child process, before any GPU call: bench.spawn_ranks).  On a one-GPU box
the two ranks share cuda:0 and exchange gradients over gloo (RCCL cannot put two ranks on one
device); everything else -- DataParallel's bucketed all-reduces, the barrier + max-over-ranks
timing, rank 0's single JSON line -- is the path the 8-GPU run takes.  The gradient averaging
follows the reference's per-rank loss scaling (layers/losses.py:34).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_one_json_line():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--cpu-sample", "0"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=170)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 512
    assert out["value"] > 0 and out["value"] == out["value"]  # finite, positive
    assert out["ms_per_step"] > 0
