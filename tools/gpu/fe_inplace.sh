#!/bin/bash
# the front-end with log2 S kept in the clip's norm slot (FE_INPLACE variant) against the
# register-resident product: config-2 bench (time + parity), then FETCH_SIZE / WRITE_SIZE per launch
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fein
for L in mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_fein.so; do
  tag=$(basename $L .so)
  for r in 1 2; do
    timeout -k 10 300 python3 tools/bench_with_lib.py $L --workload od_features --no-cpu-baseline > gpurun_out/fein/bench_${tag}_$r.json 2> gpurun_out/fein/err.log || { echo "bench rc=$?"; tail -5 gpurun_out/fein/err.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/fein/bench_${tag}_$r.json') if l.startswith('{')][0])
r=d['roofline']; p=d['parity']
print('$tag', round(d['value']), 'ms/launch', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],4), 'norm err', p['od_norm_logmel_max_abs_err'], 'zcr bad', p['zcr_count_mismatch_clips'])"
  done
  for ctr in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/fein/p_$ctr
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/fein/p_$ctr -o p -- python3 tools/bench_with_lib.py $L --workload od_features --steps 3 --warmup 0 --no-cpu-baseline --no-parity > gpurun_out/fein/p_$ctr.log 2>&1 || { echo "pmc $ctr failed"; tail -5 gpurun_out/fein/p_$ctr.log; exit 1; }
  done
  python3 tools/pmc_traffic.py od_features gpurun_out/fein/p_FETCH_SIZE gpurun_out/fein/p_WRITE_SIZE gpurun_out/fein/p_FETCH_SIZE.log > gpurun_out/fein/traffic_$tag.json || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/fein/traffic_$tag.json')); st=d['stages']['od_fe']
print('$tag traffic', {k: st[k] for k in st if 'bytes' in k or 'ratio' in k or 'per_clip' in k})"
  rm -rf gpurun_out/fein/p_*
done
