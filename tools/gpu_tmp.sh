cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2; do
  timeout -k 10 120 python tools/kbench.py --iters 30 --tag seq || exit 1
  ZMQG_CURVE_LIB=$PWD/build/libzmqg_seq_sc.so timeout -k 10 120 python tools/kbench.py --iters 30 --tag seq_sc || exit 1
  ZMQG_FRAMES_G=16 ZMQG_CURVE_LIB=$PWD/build/libzmqg_st_sc.so timeout -k 10 120 python tools/kbench.py --iters 30 --tag st_sc || exit 1
done
bash tools/variant_sweep.sh
