#!/bin/bash
# OD front-end A/B: fe_ab.sh <libA.so> <libB.so> [rounds] -- alternating bench runs (avg launch ms)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A=$1; B=$2; r=${3:-2}
for i in $(seq $r); do
  for L in $A $B; do
    timeout -k 10 200 python tools/bench_with_lib.py $L --workload od_features --no-cpu-baseline --no-parity --no-latency --steps 50 > gpurun_out/feab.log 2>&1 || { tail -20 gpurun_out/feab.log; exit 1; }
    python3 -c "
import json
l=[x for x in open('gpurun_out/feab.log') if x.startswith('{')][-1]; d=json.loads(l); print('$(basename $L)', round(d['value']), round(d['roofline']['avg_launch_ms'], 4), round(d['roofline']['frac'], 4))"
  done
done
