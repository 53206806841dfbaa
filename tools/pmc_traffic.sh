#!/bin/bash
# HBM traffic of config 2's frame kernels in both forms -- MALL-resident
# (bench.py --eager, the main line alone) and HBM-fed (tools/hbm_probe.py
# --forms bench --stream-out: 8 batches with their own buffers, decoded with
# ZMQG_OPT_STREAM_OUT as bench.py hbm_fed does) -- one rocprofv3 pass per
# counter group, kernel-trace only (MI355X_MICROARCH.md HBM section):
# FETCH_SIZE; WRITE_SIZE; the L2's memory-side request counts TCC_EA0_RDREQ /
# _RDREQ_32B / _WRREQ / _WRREQ_64B.  Then FETCH_SIZE and WRITE_SIZE over
# tools/framecopy (known byte counts, lane and cooperative shapes) to
# calibrate.  Output gpurun_out/pmct/<form>/<pass>/; tools/pmc_profiles.py
# writes profiles/pmc_traffic_config2.json stamped with the source id.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/pmct
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
EA=""
for c in TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_WRREQ TCC_EA0_WRREQ_64B; do
  grep -q "\b${c}\b" $O/counters.txt && EA="$EA ${c}_sum"
done
echo "request counters: ${EA:-none listed}"
for form in resident hbm; do
  for p in fetch write ea; do
    case $p in fetch) C=FETCH_SIZE ;; write) C=WRITE_SIZE ;; ea) C="$EA" ;; esac
    [ -z "$C" ] && continue
    mkdir -p $O/$form/$p
    if [ $form = resident ]; then
      timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/$form/$p -o pmc -- \
        python bench.py --eager --steps 3 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-host-staged --no-configs \
        --no-deployable --hbm-sets 0 > $O/$form/$p/run.log 2>&1 || { echo "$form $p failed"; tail -5 $O/$form/$p/run.log; exit 1; }
    else
      timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/$form/$p -o pmc -- \
        python tools/hbm_probe.py --variants 0 --reps 1 --forms bench --stream-out > $O/$form/$p/run.log 2>&1 || { echo "$form $p failed"; tail -5 $O/$form/$p/run.log; exit 1; }
    fi
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  t=$(echo $c | tr A-Z a-z | cut -d_ -f1)
  mkdir -p $O/cal/$t
  timeout -s KILL 60 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/cal/$t -o pmc -- \
      ./tools/bin/framecopy > $O/cal/$t/run.log 2>&1 || { echo "calibration pass $c failed"; exit 1; }
done
echo done
