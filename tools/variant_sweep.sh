#!/bin/bash
# Frame-kernel variant sweep: config-2-shaped batches
# (1 KiB frames, one session) at sizes around one wave per SIMD, every
# variant forced (ZMQG_FRAMES_G: 4, 2 = G lanes per frame, 0 = seq,
# 8 = lds, 16 = st) and the library's own choice.
cd "${GRAFT_REPO_ROOT:-.}"
for m in ${SIZES:-32768 49152 60000 65535 65536 70000 98304 131072}; do
  for g in default 4 2 0 8 16; do
    if [ $g = default ]; then
      timeout -k 10 120 python tools/kbench.py --iters 20 --msgs $m --tag "n=$m G=default" || exit 1
    else
      ZMQG_FRAMES_G=$g timeout -k 10 120 python tools/kbench.py --iters 20 --msgs $m --tag "n=$m G=$g" || exit 1
    fi
  done
done
