#!/bin/bash
# round 4 check: GPU test suite (optionally a subset first), then the od_features bench line.
#   FIRST="tests/test_gpu_range_guard.py ..."  runs those test files before the whole suite
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$FIRST" ]; then
  timeout -k 10 400 python3 -u -m pytest $FIRST -q -x --timeout 200 --timeout-method thread > gpurun_out/r4_first.log 2>&1
  rc=$?; tail -5 gpurun_out/r4_first.log; [ $rc = 0 ] || exit 1
fi
if [ -z "$NOSUITE" ]; then
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r4_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/r4_pytest.log; [ $rc = 0 ] || exit 1
fi
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload od_features --no-cpu-baseline --no-latency --steps 50 > gpurun_out/r4_fe.log 2>&1 || { tail -20 gpurun_out/r4_fe.log; exit 1; }
  grep '^{' gpurun_out/r4_fe.log | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('od_features', round(d['value']), r['avg_launch_ms'], round(r['frac'],4), d.get('parity'))"
done
