#!/bin/bash
# FE waves-per-clip A/B (default build = FE_NW 2) at 4096 and 65 536 clips, alternating builds
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_corun.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fenw_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fenw_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/fenw_tests.log | head -30; exit $rc; }
for i in 1 2; do
for n in 4096 65536; do
for L in mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_nw1.so mmla_audio_amd/ab/libmmla_nw4.so; do
  timeout -k 10 300 python3 tools/bench_with_lib.py $L --workload od_features --clips $n --no-cpu-baseline --no-parity --steps 10 > gpurun_out/fenw.log 2>&1 || { tail -20 gpurun_out/fenw.log; exit 1; }
  grep '^{' gpurun_out/fenw.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$(basename $L)', $n, round(d['value']), round(d['roofline']['frac'],4))"
done; done; done
