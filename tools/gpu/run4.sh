#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -rA -x > gpurun_out/pytest_gpu4.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "relative|PASS|FAIL|Error|passed|failed" gpurun_out/pytest_gpu4.log | head -40
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py --cpu-seconds 5 > gpurun_out/bench_od4.log 2>&1 || exit $?
echo "bench od done"; tail -1 gpurun_out/bench_od4.log | cut -c 1-2500
