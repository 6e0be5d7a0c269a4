#!/bin/bash
# A/B/n of library builds on one box: abn.sh <workload> <rounds> <lib>... (alternating runs; prints
# value and per-stage ms per run)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
wl=$1; r=$2; shift 2
for i in $(seq $r); do
  for L in "$@"; do
    timeout -k 10 300 python3 tools/bench_with_lib.py $L --workload $wl --no-cpu-baseline --no-f32 --no-parity --no-latency > gpurun_out/abn_run.log 2>&1 || { tail -20 gpurun_out/abn_run.log; exit 1; }
    grep '^{' gpurun_out/abn_run.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$(basename $L)', round(d['value']), {k:v['ms'] for k,v in d['stages'].items()})"
  done
done
