#!/bin/bash
# Conv1D zero-row change: SI GPU tests, then SI A/B against ab/libmmla_convold.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batching.py tests/test_gpu_sharded.py tests/test_gpu_range_guard.py -x -q --timeout 200 --timeout-method thread > gpurun_out/zr_tests.log 2>&1
rc=$?; tail -2 gpurun_out/zr_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/zr_tests.log | head -30; exit $rc; }
bash tools/gpu/ab.sh si_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_convold.so 3
