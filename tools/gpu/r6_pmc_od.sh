#!/bin/bash
# Round-6 checkpoint, part 4: SQ counters of the OD pipeline kernels
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/pmc_kernels.sh od_pipeline 16384 r6od > gpurun_out/pmc_r6od.log 2>&1 || { tail -20 gpurun_out/pmc_r6od.log; exit 1; }
