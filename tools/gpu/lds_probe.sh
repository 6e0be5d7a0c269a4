#!/bin/bash
# dev: LDS isolation probe between co-running workgroups of two kernels (tools/lds_probe.hip)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/lds_probe > gpurun_out/lds_probe.log 2>&1; rc=$?
cat gpurun_out/lds_probe.log; exit $rc
