#!/bin/bash
# Round-6 checkpoint, part 1: the whole GPU suite, then the PMC traffic captures bench.py reads
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/fin_pytest.log 2>&1 || { tail -30 gpurun_out/fin_pytest.log; exit 1; }
tail -3 gpurun_out/fin_pytest.log
bash tools/gpu/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || { tail -20 gpurun_out/pmc_traffic.log; exit 1; }
grep -h traffic_bytes_per_launch gpurun_out/pmc_traffic_*.json
