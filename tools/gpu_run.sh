#!/bin/bash
# One entry point for the GPU-box runs behind DESIGN.md and profiles/
# (replaces round 4's eighteen one-off tools/gpu_r4_*.sh scripts).
#
#   gpurun -- 'bash tools/gpu_run.sh MODE [ARGS]'
#
# MODE
#   suite            the whole -m gpu suite in one process, then smoke()
#   bench            the bench line with the driver's arguments (K=20, W=5)
#   prof             rocprofv3 --kernel-trace --stats of the config-2-only bench
#                    (profiles/<tag>_config2_kernel_stats.csv), then of the full
#                    bench (all configs) -- ARGS: tag (default rNN)
#   pmc              PMC passes of the config-2 bench for profiles/pmc_*_config2.json
#                    (tools/pmc_profiles.sh; summarise with tools/pmc_profiles.py)
#   ab LIB [SHAPE]   config-2 (or SHAPE = kbench args) frame kernels of library
#                    LIB against the tree's, alternating, three rounds
#   benchab LIB      the bench line of LIB against the tree's, alternating
#   zmtp             tests/test_zmtp.py, tools/zmtp_bench.py twice, a kernel trace
#   msg              per-message path: its tests, tools/bin/msg_kernel_bench
#                    (per call), tools/bin/msg_latency (round trips)
#   cfg4             config 4 as the bench runs it, each frame-kernel variant forced
#   twowave          one-lane kernels at one and two waves per SIMD over 64 MiB
#   engine           the host-adapter tests (batcher, engine hook with epoll)
#   sweep            frame kernels just above one wave per SIMD: the library's
#                    choice (k_frames_split) against k_frames_seq forced
#   pmc4             config-4 PMC passes (instruction mix, wave-cycle shares,
#                    TA/TD) of the frame kernels, encode against decode
#   settle           tools/replay_series.py: the timed replay's step time,
#                    replay after replay (clock ramp), 20- and 100-step graphs
# Every GPU step runs under its own time limit and the script stops at the
# first failure.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MODE=${1:-suite}
shift
PYTEST="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
kb() { timeout -k 10 180 python -u tools/kbench.py "$@"; }

case $MODE in
suite)
  timeout -k 10 1000 $PYTEST tests -m gpu > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
  if [ $rc -ne 0 ]; then grep -B5 -A30 "FAILED\|Error" gpurun_out/pytest_gpu.log | head -80; exit 1; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
  ;;
bench)
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err \
    || { tail -20 gpurun_out/bench.err; exit 1; }
  tail -1 gpurun_out/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['pmc_files'], {k: round(v['value'],1) for k,v in d.get('configs',{}).items()})"
  ;;
prof)
  TAG=${1:-rNN}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_c2 -o c2 --output-format csv -- \
      python3 bench.py --steps 20 --warmup 5 --no-configs --no-host-staged --no-cpu-baseline \
      > gpurun_out/prof_c2.json 2> gpurun_out/prof_c2.err || { tail -20 gpurun_out/prof_c2.err; exit 1; }
  tail -1 gpurun_out/prof_c2.json
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_all -o all --output-format csv -- \
      python3 bench.py --steps 20 --warmup 5 --no-host-staged --no-cpu-baseline \
      > gpurun_out/prof_all.json 2> gpurun_out/prof_all.err || { tail -20 gpurun_out/prof_all.err; exit 1; }
  find gpurun_out/prof_c2 gpurun_out/prof_all -name "*kernel_stats.csv"
  ;;
pmc)
  bash tools/pmc_profiles.sh || exit 1
  ;;
ab)
  A=$1; shift
  for r in 1 2 3; do
    for lib in $A libzmq_amd/libzmqg_curve.so; do
      ZMQG_CURVE_LIB=$PWD/$lib kb --tag $lib "$@" > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
      tail -1 gpurun_out/ab.log
    done
  done
  ;;
benchab)
  A=$1
  for r in 1 2; do
    for lib in $A libzmq_amd/libzmqg_curve.so; do
      ZMQG_CURVE_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
          --no-host-staged --no-configs > gpurun_out/benchab.json 2> gpurun_out/benchab.err \
          || { tail -20 gpurun_out/benchab.err; exit 1; }
      tail -1 gpurun_out/benchab.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value'],1), round(d['ms_per_step']*1000,1), round(d['roofline']['avg_launch_us'],1), round(d['roofline']['encode_main_avg_us'],1))"
    done
  done
  ;;
zmtp)
  timeout -k 10 300 $PYTEST tests/test_zmtp.py -m gpu > gpurun_out/pytest_zmtp.log 2>&1 \
    || { tail -40 gpurun_out/pytest_zmtp.log; exit 1; }
  tail -1 gpurun_out/pytest_zmtp.log
  for r in 1 2; do
    timeout -k 10 180 python -u tools/zmtp_bench.py || exit 1
  done
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/zprof -o run --output-format csv -- \
      python -u tools/zmtp_bench.py > gpurun_out/zprof.log 2>&1 || { tail -20 gpurun_out/zprof.log; exit 1; }
  find gpurun_out/zprof -name "*kernel_trace.csv" -delete
  ;;
msg)
  timeout -k 10 300 $PYTEST tests/test_gpu_msg.py tests/test_host_adapter.py -m gpu > gpurun_out/pytest_msg.log 2>&1 \
    || { tail -30 gpurun_out/pytest_msg.log; exit 1; }
  tail -1 gpurun_out/pytest_msg.log
  LD_LIBRARY_PATH=$PWD/libzmq_amd:$LD_LIBRARY_PATH timeout -k 10 120 ./tools/bin/msg_kernel_bench tree || exit 1
  timeout -k 10 120 ./tools/bin/msg_latency > gpurun_out/msg_latency.json 2>&1 || exit 1
  grep '^{' gpurun_out/msg_latency.json
  ;;
cfg4)
  for r in 1 2; do
    for g in default 0 8; do
      if [ $g = default ]; then unset ZMQG_FRAMES_G; else export ZMQG_FRAMES_G=$g; fi
      timeout -k 10 300 python bench.py --steps 5 --warmup 2 --configs 4 --no-cpu-baseline --no-host-staged 2>/dev/null \
        | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); c=d['configs']['config4']; print('G=$g', 'config4', round(c['value'],1), 'GiB/s', round(c['ms_per_step'],3), 'ms/step')" || exit 1
    done
  done
  ;;
twowave)
  for r in 1 2; do
    for g in 0 8; do
      ZMQG_FRAMES_G=$g kb --iters 30 --msgs 65536 --size 1024 --tag G$g-65536x1024 || exit 1
      ZMQG_FRAMES_G=$g kb --iters 30 --msgs 131072 --size 512 --tag G$g-131072x512 || exit 1
    done
  done
  ;;
engine)
  timeout -k 10 600 $PYTEST -s tests/test_host_adapter.py tests/test_gpu_notify.py tests/test_libzmq_interop.py \
      > gpurun_out/pytest_engine.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_engine.log
  if [ $rc -ne 0 ]; then grep -B5 -A30 "FAILED\|Error" gpurun_out/pytest_engine.log | head -60; exit 1; fi
  grep -E "^OK 4800|'msgs_per_s'" gpurun_out/pytest_engine.log || true
  ;;
sweep)
  for r in 1 2; do
    for n in 65536 65537 70000 73728 73729 81920 81921 98304; do
      kb --iters 20 --msgs $n --size 1024 --tag split-$n || exit 1
      ZMQG_FRAMES_G=0 kb --iters 20 --msgs $n --size 1024 --tag seq-$n || exit 1
    done
  done
  ;;
pmc4)
  O=gpurun_out/pmc4
  mkdir -p $O
  timeout -k 10 60 rocprofv3 --list-avail > $O/counters.txt 2>&1 || true
  p=0
  for C in "SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_INSTS_SMEM" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE GRBM_TA_BUSY" \
           "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" ; do
    p=$((p + 1))
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $PWD/$O/p$p -o pmc -- \
        python tools/kbench.py --msgs 16777216 --size 256 --sessions 1024 --sid-mod --iters 2 > $O/p$p.log 2>&1
    rc=$?
    # (an unknown counter name fails the pass at once; a kill or a crash ends the call)
    case $rc in 0) ;; 124|134|137|139) echo "pmc4 pass $p: rc $rc"; tail -5 $O/p$p.log; exit 1 ;;
                *) echo "pmc4 pass $p failed (rc $rc)"; tail -3 $O/p$p.log ;; esac
  done
  ;;
pmc4b)
  # config 4: the store ablations' counters, and VALU per frame against the
  # frame's window count (k_frames_lds forced) for the fixed per-frame part
  O=gpurun_out/pmc4b
  mkdir -p $O
  C="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES"
  for L in default abl512 abl1024 abl1536; do
    LIB=""; [ $L != default ] && LIB=$PWD/tools/bin/$L/libzmqg_curve.so
    ZMQG_CURVE_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $PWD/$O/$L -o pmc -- \
        python tools/kbench.py --msgs 16777216 --size 256 --sessions 1024 --sid-mod --iters 2 > $O/$L.log 2>&1 \
        || { echo "pmc4b $L failed"; tail -5 $O/$L.log; exit 1; }
  done
  for P in 128 192 256 384 512 768; do
    ZMQG_FRAMES_G=8 timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $PWD/$O/sz$P -o pmc -- \
        python tools/kbench.py --msgs 1048576 --size $P --sessions 1024 --sid-mod --iters 2 > $O/sz$P.log 2>&1 \
        || { echo "pmc4b size $P failed"; tail -5 $O/sz$P.log; exit 1; }
  done
  # (only the counter summaries come back: gpurun_out is capped)
  find $O -name "*kernel_trace.csv" -delete
  find $O -name "*agent_info.csv" -delete
  ;;
probe)
  # the per-message floor: one launch per request (launch_floor) against a
  # resident kernel polling a doorbell in host memory (resident_probe)
  timeout -k 10 120 ./tools/bin/launch_floor || exit 1
  timeout -k 10 60 ./tools/bin/resident_probe || exit 1
  ;;
hookbench)
  # the batched adapter end to end: two epoll I/O threads, socketpairs,
  # GPU encode on one side and decode on the other (tests/host/test_engine_hook.cpp bench)
  for a in "16 20000 1024" "64 5000 1024" "256 1500 1024" "64 20000 256"; do
    timeout -k 10 90 ./tools/bin/engine_hook_bench bench $a || exit 1
  done
  ;;
interop)
  timeout -k 10 600 $PYTEST -s tests/test_libzmq_interop.py > gpurun_out/pytest_interop.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_interop.log
  if [ $rc -ne 0 ]; then grep -B5 -A30 "FAILED\|Error" gpurun_out/pytest_interop.log | head -60; exit 1; fi
  grep -E "'msgs_per_s'|'gamma'" gpurun_out/pytest_interop.log || true
  ;;
settle)
  timeout -k 10 180 python -u tools/replay_series.py --reps 60 || exit 1
  timeout -k 10 180 python -u tools/replay_series.py --reps 30 --steps 100 || exit 1
  ;;
*)
  echo "unknown mode $MODE"; exit 2
  ;;
esac
