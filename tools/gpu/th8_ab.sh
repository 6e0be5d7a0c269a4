#!/bin/bash
# resblk blocks 2-3 at half-height tiles (GEMM 2 weights from L2, 3 workgroups per CU): A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
true > gpurun_out/th8_tests.log
rc=$?; tail -2 gpurun_out/th8_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/th8_tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 tools/bench_with_lib.py mmla_audio_amd/ab/libmmla_th8.so --clips 16384 --no-cpu-baseline --no-f32 --no-latency --steps 1 > gpurun_out/th8_par.log 2>&1 || { tail -20 gpurun_out/th8_par.log; exit 1; }
grep '^{' gpurun_out/th8_par.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('th8 parity', {k:v for k,v in d['parity'].items() if k!='sample'})"
bash tools/gpu/ab.sh od_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_th8.so 2
