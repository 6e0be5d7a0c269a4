#!/bin/bash
# resblk variants: OD parity tests on the product build, then per-kernel rocprof A/B and pipeline A/Bs
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batching.py tests/test_gpu_range_guard.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rb_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rb_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/rb_tests.log | head; exit $rc; }
bash tools/gpu/prof_ab.sh od_pipeline mmla_audio_amd/ab/libmmla_base.so mmla_audio_amd/libmmla.so 2>&1 | grep -E "==|resblk" || exit 1
bash tools/gpu/prof_ab.sh od_pipeline mmla_audio_amd/ab/libmmla_w2l2.so mmla_audio_amd/libmmla.so 2>&1 | grep -E "==|resblk" || exit 1
bash tools/gpu/ab.sh od_pipeline mmla_audio_amd/ab/libmmla_base.so mmla_audio_amd/libmmla.so 2 || exit 1
