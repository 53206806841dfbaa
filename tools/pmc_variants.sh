#!/bin/bash
# PMC passes (tools/pmc_frames.sh) over config 2 for the default frame kernel
# and a forced variant: tools/pmc_variants.sh G
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/pmc_frames.sh gpurun_out/pmc_default --iters 5 || exit 1
ZMQG_FRAMES_G=$1 bash tools/pmc_frames.sh gpurun_out/pmc_g$1 --iters 5 || exit 1
python3 tools/pmc_summary2.py gpurun_out/pmc_default
python3 tools/pmc_summary2.py gpurun_out/pmc_g$1
