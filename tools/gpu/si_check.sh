#!/bin/bash
# SI front-end: GPU parity tests, then v1 vs v2 throughput on config 4
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "si_" --timeout 120 --timeout-method thread > gpurun_out/si_tests.log 2>&1
rc=$?; tail -5 gpurun_out/si_tests.log; [ $rc -eq 0 ] || exit $rc
for impl in 2 1; do
  MMLA_SI_FE_IMPL=$impl timeout -k 10 300 python3 bench.py --workload si_pipeline --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/si_bench_$impl.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/si_bench_$impl.log') if l.startswith('{')][0]);print('impl $impl', round(d['value']), 'clips/s', d['stages'])"
done
