#!/bin/bash
# resblk GEMM-1 weight layout: GPU suite, then SI and OD A/B against ab/libmmla_rbold.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rb_tests.log 2>&1
rc=$?; tail -2 gpurun_out/rb_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/rb_tests.log | head -30; exit $rc; }

bash tools/gpu/ab.sh od_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_rbold.so 2
