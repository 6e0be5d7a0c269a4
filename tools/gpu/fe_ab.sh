#!/bin/bash
# FE change check: GPU suite, then the front-end bench at 4096 (config 2) and 65 536 clips
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fe_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fe_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/fe_tests.log | head -30; exit $rc; }
for n in 4096 65536; do
  timeout -k 10 300 python3 bench.py --workload od_features --clips $n --no-cpu-baseline --steps 10 > gpurun_out/fe_$n.log 2>&1 || { tail -20 gpurun_out/fe_$n.log; exit 1; }
  grep '^{' gpurun_out/fe_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, d['value'], d['roofline']['frac'], d.get('parity'))"
done
