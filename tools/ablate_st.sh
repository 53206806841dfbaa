#!/bin/bash
# k_frames_st diagnostics at config 2 (65,536 x 1 KiB): phase stamps
# (build/st_stamps), kernel timings of seq and st, timing ablations
# (build/libzmqg_st<V>.so = -DZMQG_ST_ABLATE=V, curve_frames_st.hpp, st
# forced; outputs not checked), and one PMC pass of wave-cycle shares per
# variant.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -x build/st_stamps ]; then timeout -k 10 60 build/st_stamps > gpurun_out/st_stamps.log 2>&1 || { cat gpurun_out/st_stamps.log; exit 1; }; cat gpurun_out/st_stamps.log; fi
timeout -k 10 120 python tools/kbench.py --iters 30 --tag seq || exit 1
ZMQG_FRAMES_G=16 timeout -k 10 120 python tools/kbench.py --iters 30 --tag st || exit 1
for v in ${ABL:-1 2 4 8 16 32 48 15}; do
  [ -f build/libzmqg_st$v.so ] || continue
  ZMQG_FRAMES_G=16 ZMQG_CURVE_LIB=$PWD/build/libzmqg_st$v.so timeout -k 10 120 python tools/kbench.py --iters 30 --tag st_ab$v || exit 1
done
C="SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
for g in ${PMCG:-0 16}; do
  O=gpurun_out/pmc_g$g
  mkdir -p $O
  ZMQG_FRAMES_G=$g timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $PWD/$O -o pmc -- \
      python tools/kbench.py --iters 3 --tag pmc$g > $O/run.log 2>&1 || { echo "pmc pass $g failed"; tail -5 $O/run.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections, os
for g in os.environ.get("PMCG", "0 16").split():
    f = glob.glob(f"gpurun_out/pmc_g{g}/**/pmc_counter_collection.csv", recursive=True)
    if not f:
        print("no pmc file", g); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if "k_frames" not in k: continue
        kk = ("dec" if "ILb1E" in k else "enc") + ("_st" if "frames_st" in k else "_seq" if "frames_seq" in k else "_other")
        acc[kk][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(kk, r["Counter_Name"])] += 1
    for kk, d in sorted(acc.items()):
        n = cnt[(kk, "SQ_WAVE_CYCLES")] or 1
        wc = d["SQ_WAVE_CYCLES"] or 1
        print(g, kk, "launches", n, " ".join(f"{c}={d[c]/n:.3g}" for c in sorted(d)),
              "| valu%", round(100 * d["SQ_ACTIVE_INST_VALU"] / wc, 1), "wait%", round(100 * d["SQ_WAIT_ANY"] / wc, 1),
              "stall%", round(100 * d["SQ_WAIT_INST_ANY"] / wc, 1), "lds_stall%", round(100 * d["SQ_WAIT_INST_LDS"] / wc, 1))
PY
