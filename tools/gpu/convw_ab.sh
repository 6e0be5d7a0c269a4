#!/bin/bash
# conv_h3 weight layout: GPU suite, then SI and OD A/B against ab/libmmla_convold.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/cw_tests.log 2>&1
rc=$?; tail -2 gpurun_out/cw_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/cw_tests.log | head -30; exit $rc; }
bash tools/gpu/ab.sh si_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_convold.so 2 || exit 1
bash tools/gpu/ab.sh od_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_convold.so 1
