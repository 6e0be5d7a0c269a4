#!/bin/bash
# full GPU suite, then the default bench line (OD pipeline, CPU baseline, f32 leg, parity sample)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r2_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/r2_tests.log | head -30; exit $rc; }
timeout -k 10 600 python3 bench.py ${BENCH_ARGS} > gpurun_out/r2_bench.log 2>&1 || { tail -30 gpurun_out/r2_bench.log; exit 1; }
grep '^{' gpurun_out/r2_bench.log > gpurun_out/r2_bench.json
python3 -c "
import json;d=json.load(open('gpurun_out/r2_bench.json'))
print('value',d['value'],'ms/step',d['ms_per_step'],'roof',d['roofline']['frac'],'mb',d['config']['microbatch'])
print('f32',d['precision_f32'] and {k:d['precision_f32'][k] for k in ('value','argmax_differs_from_f16x3')})
print('parity',d['parity']); print('cpu',d['cpu_baseline'] and d['cpu_baseline']['modes'])
print('fe',d['fe'] and d['fe']['clips_per_s'], 'range ok', d['range_guard_ok'])"
