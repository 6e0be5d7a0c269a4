#!/bin/bash
# conv_h3 register budgets: parity/batching tests, then SI and OD A/B against ab/libmmla_minw2.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batching.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mw_tests.log 2>&1
rc=$?; tail -2 gpurun_out/mw_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/mw_tests.log | head -30; exit $rc; }
bash tools/gpu/ab.sh si_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_minw2.so 2 || exit 1
bash tools/gpu/ab.sh od_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_minw2.so 2
