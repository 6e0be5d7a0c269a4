#!/bin/bash
# resblk GEMM-2 weights: GPU suite on the default build (conv(4,1) weights now in fragment order,
# copied to LDS), the RB_W2LDS=0 variant's parity on the bench sample, then an OD A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/w2_tests.log 2>&1
rc=$?; tail -2 gpurun_out/w2_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/w2_tests.log | head -30; exit $rc; }
timeout -k 10 300 python3 tools/bench_with_lib.py mmla_audio_amd/ab/libmmla_w2l2.so --clips 16384 --no-cpu-baseline --no-f32 --no-latency --steps 1 > gpurun_out/w2_par.log 2>&1 || { tail -20 gpurun_out/w2_par.log; exit 1; }
grep '^{' gpurun_out/w2_par.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('w2l2 parity', {k:v for k,v in d['parity'].items() if k!='sample'})"
bash tools/gpu/ab.sh od_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_w2l2.so 2
