#!/bin/bash
# conv XCD remap: GPU tests, then OD + SI A/B against ab/libmmla_noxcd.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/xcd_tests.log 2>&1
rc=$?; tail -2 gpurun_out/xcd_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/xcd_tests.log | head -30; exit $rc; }
bash tools/gpu/ab.sh od_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_noxcd.so 2 && bash tools/gpu/ab.sh si_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_noxcd.so 1
for i in 1 2; do
for L in mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_feold.so; do
  timeout -k 10 300 python3 tools/bench_with_lib.py $L --workload od_features --no-cpu-baseline --steps 10 > gpurun_out/fe_ab.log 2>&1 || { tail -20 gpurun_out/fe_ab.log; exit 1; }
  grep '^{' gpurun_out/fe_ab.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$(basename $L)', 'od_features', round(d['value']), round(d['roofline']['frac'],4), d['parity'].get('od_norm_logmel_max_abs_err'))"
done; done
