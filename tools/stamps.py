#!/usr/bin/env python3
"""Phase breakdown of the body kernel from a ZMQG_STAMPS build (diagnostic).
Stamps (s_memtime ticks, relative to tile start): 1 setup done, 2 phase-0
input landed in LDS, 3 phase-0 compute done, 4 phase-0 stores issued,
5 phase 1 (DMA, compute, stores) done, 6 finish done."""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = os.path.join(ROOT, "tools", "bin", "libzmqg_curve_stamps.so")
os.environ["ZMQG_CURVE_LIB"] = lib
sys.argv = [sys.argv[0], "--iters", "1"] + sys.argv[1:]
sys.path.insert(0, ROOT)
# run one kbench step set in-process, then read stamps
import runpy  # noqa: E402
runpy.run_path(os.path.join(ROOT, "tools", "kbench.py"), run_name="__main__")
L = ctypes.CDLL(lib)
buf = (ctypes.c_ulonglong * (8 * 16384))()
cnt = ctypes.c_uint32(0)
assert L.zmqg_debug_stamps(buf, 16384, ctypes.byref(cnt)) == 0
a = np.frombuffer(buf, np.uint64)[: cnt.value * 8].reshape(-1, 8)[:, :7].astype(np.float64)
print("records", cnt.value)
names = ["wait", "window0", "setupnext", "window1", "stores", "finish"]
d = np.diff(a, axis=1)
for k, nme in enumerate(names):
    print(f"  {nme:8s} mean {d[:, k].mean():9.0f}  p50 {np.median(d[:, k]):9.0f}  p90 {np.percentile(d[:, k], 90):9.0f} ticks")
print(f"  total    mean {a[:, 6].mean():9.0f}")
