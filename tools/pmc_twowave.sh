#!/bin/bash
# Round 4: why a second wave per SIMD does not help -- per-launch PMC of
# k_frames_seq at one wave per SIMD (65,536 x 1 KiB) and two (131,072 x
# 512 B, the same bytes), one rocprofv3 pass per counter group
# (tools/pmc_twowave.py summarises).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc2w
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"
P2="TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE GRBM_TA_BUSY"
P3="TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum"
P4="TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum"
for wl in "65536 1024" "131072 512"; do
  set -- $wl
  k=1
  for pass in "$P1" "$P2" "$P3" "$P4"; do
    ZMQG_FRAMES_G=0 timeout -s KILL 90 rocprofv3 --pmc $pass -d gpurun_out/pmc2w/n$1_p$k -o c --output-format csv -- python3 tools/kbench.py --msgs $1 --size $2 --iters 5 > gpurun_out/pmc2w/n$1_p$k.log 2>&1 || { tail -5 gpurun_out/pmc2w/n$1_p$k.log; exit 1; }
    k=$((k+1))
  done
done
python3 tools/pmc_twowave.py gpurun_out/pmc2w
