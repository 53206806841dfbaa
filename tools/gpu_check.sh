#!/bin/bash
# Full GPU test suite, then a default bench run (log under gpurun_out/chk).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/chk
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/chk/pytest.log 2>&1 || { tail -40 gpurun_out/chk/pytest.log; exit 1; }
tail -1 gpurun_out/chk/pytest.log
timeout -k 10 400 python bench.py > gpurun_out/chk/bench.log 2>&1 || { tail -20 gpurun_out/chk/bench.log; exit 1; }
tail -1 gpurun_out/chk/bench.log > gpurun_out/chk/bench.json
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/chk/bench.json"))
h = d["hbm_fed"]
print("main", round(d["value"], 1), "dec_us", round(d["roofline"]["avg_launch_us"], 1), "frac", round(d["roofline"]["frac"], 3))
print("hbm", round(h["value"], 1), "enc", round(h["encode_us"], 1), "dec", round(h["decode_us"], 1))
print("configs", {k: round(v["value"], 1) for k, v in d.get("configs", {}).items()})
print("host", {k: (v.get("value") if isinstance(v, dict) else v) for k, v in d.get("host_paths", {}).items()})
print("cpu", d.get("cpu_baseline", {}).get("value"), d.get("cpu_baseline", {}).get("kind"))
PY
