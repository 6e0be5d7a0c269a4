#!/bin/bash
# front-end A/B on one box: the product library (0), FE3_SKIP timing builds ab/libmmla_skip<v>.so and
# any other ab/libmmla_<name>.so named in SKIPS (e.g. SKIPS="0 prev 32")
cd $GRAFT_REPO_ROOT
for v in ${SKIPS:-0 1 2 4 8 16}; do
  case $v in
    0) lib=mmla_audio_amd/libmmla.so;;
    [0-9]*) lib=mmla_audio_amd/ab/libmmla_skip$v.so;;
    *) lib=mmla_audio_amd/ab/libmmla_$v.so;;
  esac
  timeout -k 10 200 python tools/bench_with_lib.py $lib --workload od_features --no-cpu-baseline --no-parity --no-latency --steps 50 > gpurun_out/skip$v.log 2>&1 || exit 1
  python3 -c "
import json
l=[x for x in open('gpurun_out/skip$v.log') if x.startswith('{')][-1]; d=json.loads(l); print('skip $v', d['roofline']['avg_launch_ms'])"
done
