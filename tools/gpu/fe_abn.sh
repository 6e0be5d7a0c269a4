#!/bin/bash
# front-end A/B/n on the config-2 line: fe_abn.sh <rounds> <lib>...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
r=$1; shift
for i in $(seq $r); do
  for L in "$@"; do
    timeout -k 10 200 python tools/bench_with_lib.py $L --workload od_features --no-cpu-baseline --no-parity --no-latency --steps 50 > gpurun_out/feabn.log 2>&1 || { tail -20 gpurun_out/feabn.log; exit 1; }
    python3 -c "
import json
l=[x for x in open('gpurun_out/feabn.log') if x.startswith('{')][-1]; d=json.loads(l); print('$(basename $L)', round(d['value']), round(d['roofline']['avg_launch_ms'], 4), round(d['roofline']['frac'], 4))"
  done
done
