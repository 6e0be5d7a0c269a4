#!/bin/bash
# A/B of one library under two environments on one box: env_ab.sh <workload> "<envA>" "<envB>" [rounds]
# e.g. env_ab.sh od_pipeline "MMLA_NO_SPLIT_ACT=1" "MMLA_NO_SPLIT_ACT=0" 2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
wl=$1; A=$2; B=$3; r=${4:-2}
for i in $(seq $r); do
  for E in "$A" "$B"; do
    env $E timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline --no-f32 --no-parity > gpurun_out/envab_run.log 2>&1 || { tail -20 gpurun_out/envab_run.log; exit 1; }
    grep '^{' gpurun_out/envab_run.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$E', round(d['value']), {k:v['ms'] for k,v in d['stages'].items()})"
  done
done
