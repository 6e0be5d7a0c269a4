#!/bin/bash
# resblk blocks 2-3 layout A/B: parity of each variant (bench sample vs the float64 oracle), then timing
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in mmla_audio_amd/ab/libmmla_rb3.so mmla_audio_amd/ab/libmmla_rb3r.so mmla_audio_amd/ab/libmmla_rbr.so; do
  timeout -k 10 300 python3 tools/bench_with_lib.py $L --workload od_pipeline --no-cpu-baseline --no-f32 --no-latency --steps 1 --warmup 1 > gpurun_out/rbp.log 2>&1 || { tail -20 gpurun_out/rbp.log; exit 1; }
  grep '^{' gpurun_out/rbp.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());p=d['parity'];print('$(basename $L)', 'logp err', p['logp_max_abs_err'], 'argmax', p['argmax_agree'], p['argmax_disagree_non_tie'])"
done
bash tools/gpu/abn.sh od_pipeline 2 mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_rb3.so mmla_audio_amd/ab/libmmla_rb3r.so mmla_audio_amd/ab/libmmla_rbr.so
