#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rA -k "layerwise or od_forward" -s > gpurun_out/pytest_gpu2.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "relative|PASS|FAIL|Error|error" gpurun_out/pytest_gpu2.log | head -30
exit 0
