#!/bin/bash
# GPU suite + the front-end line, its rocprof stats and SQ counters (after a front-end-only change)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/fin_pytest.log 2>&1 || { tail -30 gpurun_out/fin_pytest.log; exit 1; }
tail -1 gpurun_out/fin_pytest.log
timeout -k 10 600 python3 -u bench.py --workload od_features > gpurun_out/bench_fe.json.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_fe.json.log > gpurun_out/bench_fe.json
WL=od_features TAG=fe BENCH_ARGS="--no-latency" bash tools/gpu/prof_line.sh > gpurun_out/prof_fe_line.log 2>&1 || exit 1
bash tools/gpu/pmc_kernels.sh od_features 4096 r3fe > gpurun_out/pmc_fe.log 2>&1 || exit 1
python3 -c "
import json
d=json.load(open('gpurun_out/bench_fe.json')); r=d['roofline']; print('fe', round(d['value']), r['avg_launch_ms'], r['frac'], d['parity'])"
