#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rA > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --clips 4096 --steps 2 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_small.log 2>&1
rc=$?
echo "bench rc=$rc"
tail -5 gpurun_out/bench_small.log
exit $rc
