#!/bin/bash
# one-call check of a library change: GPU suite, then A/B against a reference build ($1) on the
# front-end line and the OD pipeline line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
REF=${1:-mmla_audio_amd/ab/libmmla_head.so}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cc_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/cc_pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/cc_pytest.log | head -20; exit 1; }
[ -n "$FE_AB" ] && { bash tools/gpu/fe_ab.sh $REF mmla_audio_amd/libmmla.so 2 || exit 1; }
bash tools/gpu/ab.sh od_pipeline $REF mmla_audio_amd/libmmla.so 2 || exit 1
bash tools/gpu/ab.sh si_pipeline $REF mmla_audio_amd/libmmla.so 2 || exit 1
