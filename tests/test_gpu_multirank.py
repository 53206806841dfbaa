"""bench.py --gpus 2 on the GPU box: the launcher starts two ranks (torchrun,
127.0.0.1), each rank runs the config-2 step on its GPU -- ranks share a
device when the box has fewer GPUs than ranks -- config 5 splits one batch
over the ranks with shard.partition (strong scaling, sum over ranks), and
rank 0 prints exactly one line, with n_gpus = 2 and max-over-ranks timing.
The multi-process path the driver's 8-GPU scaling run takes, on real
kernels rather than the gloo tests' CPU stand-ins."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_config2_and_strong_config5():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--no-cpu-baseline", "--no-host-staged", "--configs", "5"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["scaling"] == "weak"
    assert d["config"]["parallelism"].startswith("frame-sharded x2")
    assert d["value"] > 0 and d["msgs_per_s"] > 0
    c5 = d["configs"]["config5"]
    assert c5["scaling"] == "strong" and c5["frames_per_gpu"] == 512 and c5["value"] > 0
