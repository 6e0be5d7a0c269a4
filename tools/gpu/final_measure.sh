#!/bin/bash
# GPU suite, PMC traffic first (bench.py reads the committed captures), then the 4-workload bench suite + OD rocprof
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/fm_pytest.log 2>&1 || { tail -30 gpurun_out/fm_pytest.log; exit 1; }
tail -1 gpurun_out/fm_pytest.log
bash tools/gpu/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || exit $?
cp gpurun_out/pmc_traffic_*.json profiles/
bash tools/gpu/bench_all.sh || exit $?
