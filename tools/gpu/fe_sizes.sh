#!/bin/bash
# front-end line at config 2 (4096 clips) and at 65 536 clips, v3 (default) and v2 (MMLA_OD_FE_V2=1)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 4096 65536; do
  for v in 0 1; do
    MMLA_OD_FE_V2=$v timeout -k 10 300 python3 bench.py --workload od_features --clips $n --no-cpu-baseline --no-parity --no-latency --steps 50 > gpurun_out/fes.log 2>&1 || { tail -20 gpurun_out/fes.log; exit 1; }
    grep '^{' gpurun_out/fes.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('clips $n v2=$v', round(d['value']), round(r['avg_launch_ms'],4), round(r['frac'],4))"
  done
done
