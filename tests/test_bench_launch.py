"""bench.py --gpus N outside torchrun starts N ranks itself (a fresh child
torch.distributed.run, before any GPU call).  --dry-run stops each rank after
one gloo barrier, so the launch is checked on a CPU host."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_launches_two_ranks():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--msgs", "64"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines, dec, pos = [], json.JSONDecoder(), 0
    while True:  # every JSON object in the output, however the ranks' lines fell
        pos = r.stdout.find("{", pos)
        if pos < 0:
            break
        obj, pos = dec.raw_decode(r.stdout, pos)
        lines.append(obj)
    assert sorted(d["rank"] for d in lines) == [0, 1], r.stdout
    assert all(d["world"] == 2 and d["dry_run"] for d in lines)


def test_bench_single_rank_dry_run():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["world"] == 1 and d["rank"] == 0
