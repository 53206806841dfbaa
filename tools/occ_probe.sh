cd $GRAFT_REPO_ROOT
for m in 65536 131072 262144; do
  timeout -k 10 120 python tools/kbench.py --iters 20 --msgs $m --tag seq-$m || exit 1
  ZMQG_FRAMES_G=8 timeout -k 10 120 python tools/kbench.py --iters 20 --msgs $m --tag lds-$m || exit 1
done
