#!/bin/bash
# Round-6 counters at HEAD: SQ issue/stall picture of the OD and SI pipelines (-> profiles/r6_pmc_*)
# and the PMC traffic captures bench.py reads (profiles/pmc_traffic_*.json)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/pmc_kernels.sh si_pipeline 65536 r6si > gpurun_out/pmc_r6si.log 2>&1 || { tail -20 gpurun_out/pmc_r6si.log; exit 1; }
bash tools/gpu/pmc_kernels.sh od_pipeline 16384 r6od > gpurun_out/pmc_r6od.log 2>&1 || { tail -20 gpurun_out/pmc_r6od.log; exit 1; }
bash tools/gpu/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || { tail -20 gpurun_out/pmc_traffic.log; exit 1; }
grep -h traffic_bytes_per_launch gpurun_out/pmc_traffic_*.json
