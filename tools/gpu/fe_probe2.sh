#!/bin/bash
# OD front-end (no packed FP32): phase timeline and PMC issue picture
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/fe_timeline.py > gpurun_out/fe_timeline.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/fe_timeline.log
bash tools/gpu/pmc_fe.sh
