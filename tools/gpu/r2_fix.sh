#!/bin/bash
# co-run matrix of the product build (front-end next to the network kernels), the full GPU suite,
# and front-end throughput
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/corun_diag7.py > gpurun_out/corun7.log 2>&1 || { tail -20 gpurun_out/corun7.log; exit 1; }
grep -v amdgpu.ids gpurun_out/corun7.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite.log 2>&1
rc=$?; tail -3 gpurun_out/suite.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/suite.log | head; exit $rc; }
for n in 4096 65536; do
  timeout -k 10 300 python3 bench.py --workload od_features --clips $n --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fe_$n.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/fe_$n.log') if l.startswith('{')][0]);r=d['roofline'];print($n,'clips/s',round(d['value']),'launch ms',round(r['avg_launch_ms'],4),'frac',round(r['frac'],4))"
done
