#!/bin/bash
# full GPU test suite, then short OD / SI pipeline benches with per-stage times
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quick_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/quick_tests.log | head; exit $rc; }
for wl in od_pipeline si_pipeline; do
  timeout -k 10 300 python3 bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/quick_$wl.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/quick_$wl.log') if l.startswith('{')][0]);print('$wl', round(d['value']), 'clips/s', {k:(v['ms'],v.get('TFLOP/s',v.get('GB/s'))) for k,v in d['stages'].items()})"
done
