#!/bin/bash
# round 4 end: the VALU rate probe, then round_final.sh (GPU suite, PMC traffic, the four bench
# lines + rocprof stats of the OD / SI / FE lines)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 90 ./tools/ubench/valu_rates 2100 > gpurun_out/valu_rates.txt 2>&1 || exit 1
cat gpurun_out/valu_rates.txt
bash tools/gpu/round_final.sh
