#!/bin/bash
# HEAD check: full GPU suite, smoke(), default bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/hc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/hc_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/hc_tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/hc_smoke.log 2>&1 || { tail -20 gpurun_out/hc_smoke.log; exit 1; }
tail -1 gpurun_out/hc_smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/hc_bench.log 2>&1 || { tail -20 gpurun_out/hc_bench.log; exit 1; }
grep '^{' gpurun_out/hc_bench.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['roofline']['frac'], d['parity']['argmax_agree'], d['parity']['prob_max_abs_err'])"
