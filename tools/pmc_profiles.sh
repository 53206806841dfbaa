#!/bin/bash
# All PMC passes behind profiles/pmc_*_config2.json for the current build:
# VALU counts (tools/pmc_valu_bench.sh) and HBM traffic with its calibration
# (tools/pmc_traffic.sh); tools/pmc_profiles.py writes the JSON files.
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/pmc_valu_bench.sh > /dev/null || exit 1
bash tools/pmc_traffic.sh || exit 1
