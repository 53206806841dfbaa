#!/bin/bash
# Round 4, first GPU pass: the Salsa20 issue-order microbenchmark, the new
# tests, the per-message latency, then the skewed-Salsa20 library build
# (build/libzmqg_skew1.so / skew2.so, -DZMQG_SALSA_SKEW=1 / 2) against the default: parity
# of the frame/body kernels on it, and kernel timings (config 2 frame
# kernels; 64 KiB frames through the body kernel), two rounds interleaved.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 120 ./build/salsa_sched > gpurun_out/salsa_sched.json 2>&1 || { cat gpurun_out/salsa_sched.json; exit 1; }
cat gpurun_out/salsa_sched.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_msg.py tests/test_gpu_session_batch.py tests/test_host_adapter.py tests/test_gpu_multirank.py tests/test_gpu_verify_first.py tests/test_gpu_bench_batches.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
echo "pytest_new rc=$?"; tail -30 gpurun_out/pytest_new.log
timeout -k 10 120 ./build/msg_latency > gpurun_out/msg_latency.json 2>&1; echo "msg_latency rc=$?"; cat gpurun_out/msg_latency.json
for v in 1 2; do
  ZMQG_CURVE_LIB=$PWD/build/libzmqg_skew$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_timed_path.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_skew$v.log 2>&1
  echo "pytest_skew$v rc=$?"; tail -5 gpurun_out/pytest_skew$v.log
done
for r in 1 2; do
  for lib in default skew1 skew2; do
    L=""; [ $lib != default ] && L=$PWD/build/libzmqg_$lib.so
    ZMQG_CURVE_LIB=$L timeout -k 10 120 python tools/kbench.py --iters 30 --tag $lib || exit 1
    ZMQG_CURVE_LIB=$L timeout -k 10 120 python tools/kbench.py --iters 10 --msgs 2048 --size 65536 --tag $lib-64k || exit 1
    ZMQG_CURVE_LIB=$L timeout -k 10 120 python tools/kbench.py --iters 10 --msgs 131072 --size 1024 --tag $lib-131k || exit 1
    ZMQG_CURVE_LIB=$L timeout -k 10 120 python tools/kbench.py --iters 5 --msgs 1048576 --size 256 --sessions 1024 --tag $lib-1Mx256 || exit 1
  done
done
