#!/bin/bash
# precision/range tests after a conv kernel change, then OD + SI bench lines (stage tables in the logs)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_range_guard.py tests/test_gpu_fullsize.py tests/test_gpu_batching.py -x -v --timeout 300 --timeout-method thread > gpurun_out/conv_tests.log 2>&1
rc=$?; tail -4 gpurun_out/conv_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/conv_tests.log | head -30; exit $rc; }
for w in od_pipeline si_pipeline; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --no-f32 > gpurun_out/conv_bench_$w.log 2>&1 || { tail -30 gpurun_out/conv_bench_$w.log; exit 1; }
  grep '^{' gpurun_out/conv_bench_$w.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$w',d['value'],d['ms_per_step'],d['roofline']['frac'],d['parity'] and {k:d['parity'][k] for k in ('prob_max_abs_err','argmax_disagree_non_tie')})"
done
