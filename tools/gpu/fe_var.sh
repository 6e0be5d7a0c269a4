#!/bin/bash
# front-end change: the OD GPU tests (parity, batching, drop-in, corun), then the config-2 line A/B
# against a reference build ($1)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fv_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/fv_pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/fv_pytest.log | head -20; exit 1; }
bash tools/gpu/fe_ab.sh $1 mmla_audio_amd/libmmla.so 3 || exit 1
bash tools/gpu/ab.sh od_pipeline $1 mmla_audio_amd/libmmla.so 1 || exit 1
