#!/bin/bash
# OD front-end probe: throughput vs batch size, v2 phase timeline, PMC issue picture
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 4096 16384 65536; do
  timeout -k 10 300 python3 bench.py --workload od_features --clips $n --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fe_$n.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/fe_$n.log') if l.startswith('{')][0]);r=d['roofline'];print($n,'clips/s',round(d['value']),'launch ms',round(r['avg_launch_ms'],4),'frac',round(r['frac'],4))"
done
timeout -k 10 300 python3 tools/fe_timeline.py > gpurun_out/fe_timeline.log 2>&1 || exit $?
cat gpurun_out/fe_timeline.log
bash tools/gpu/pmc_fe.sh
