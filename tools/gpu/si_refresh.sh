#!/bin/bash
# GPU suite + SI pipeline bench, rocprof stats and PMC traffic (after an SI change)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/si_pytest.log 2>&1 || { tail -30 gpurun_out/si_pytest.log; exit 1; }
tail -1 gpurun_out/si_pytest.log
timeout -k 10 600 python3 bench.py --workload si_pipeline > gpurun_out/bench_si.json.log 2>&1 || exit $?
grep '^{' gpurun_out/bench_si.json.log > gpurun_out/bench_si.json
bash tools/gpu/prof_si.sh | head -8 || exit $?
bash tools/gpu/pmc_traffic.sh > gpurun_out/pmc_traffic.log 2>&1 || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/bench_si.json')); print('si', round(d['value']), d['roofline'])"
