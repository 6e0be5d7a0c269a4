#!/bin/bash
# Round-end measurement, part 2: PMC traffic of the three roofline stages (bench.py reads the
# committed captures) and the SQ issue/stall picture of the OD pipeline kernels
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || { tail -20 gpurun_out/pmc_traffic.log; exit 1; }
grep -h traffic_bytes_per_launch gpurun_out/pmc_traffic_*.json | head
bash tools/gpu/pmc_kernels.sh od_pipeline 16384 r3od > gpurun_out/pmc_r3od.log 2>&1 || { tail -20 gpurun_out/pmc_r3od.log; exit 1; }
head -40 gpurun_out/pmc_r3od_summary.txt
