#!/bin/bash
# GPU tests + OD pipeline kernel profile (per-kernel A/B within one box)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/quick_tests.log | head; exit $rc; }
bash tools/gpu/prof_od.sh
