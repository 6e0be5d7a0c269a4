#!/bin/bash
# the GPU test suite, then (optional) the default bench line; every GPU step under its own limit
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1 || { echo "suite rc=$?"; tail -30 gpurun_out/suite.log; exit 1; }
tail -3 gpurun_out/suite.log
if [ "$1" = "bench" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/bench_od.json 2> gpurun_out/bench_od.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_od.err; exit 1; }
  cat gpurun_out/bench_od.json
fi
