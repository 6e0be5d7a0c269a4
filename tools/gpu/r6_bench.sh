#!/bin/bash
# Round-6 checkpoint, part 2: the SI PMC traffic capture, then the bench lines + OD rocprof stats
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
PMC_WL=si_pipeline bash tools/gpu/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || { tail -20 gpurun_out/pmc_traffic.log; exit 1; }
cp gpurun_out/pmc_traffic_si_pipeline.json profiles/
bash tools/gpu/bench_all.sh
