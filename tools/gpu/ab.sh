#!/bin/bash
# A/B of library builds on one box: ab.sh <workload> <libA.so> <libB.so> [rounds]
# (alternating runs so box drift hits both; prints value and the conv stage per run)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
wl=$1; A=$2; B=$3; r=${4:-2}
for i in $(seq $r); do
  for L in $A $B; do
    timeout -k 10 300 python3 tools/bench_with_lib.py $L --workload $wl --no-cpu-baseline --no-f32 --no-parity > gpurun_out/ab_run.log 2>&1 || { tail -20 gpurun_out/ab_run.log; exit 1; }
    grep '^{' gpurun_out/ab_run.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$(basename $L)', round(d['value']), {k:v['ms'] for k,v in d['stages'].items()})"
  done
done
