#!/bin/bash
# round 4 measurement batch: GPU tests, front-end A/B + phase-skip timings, conv staging A/B,
# SI pipeline PMC summary.  Steps chained: the first failure ends the call.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
FIRST="tests/test_gpu_range_guard.py tests/test_gpu_fe_persistent.py tests/test_gpu_parity.py tests/test_gpu_dropin.py" \
  NOSUITE=$NOSUITE bash tools/gpu/r4_check.sh || exit 1
SKIPS="${SKIPS:-0 prev 0 prev 32 64 128 224}" bash tools/gpu/fe_phase_skip.sh || exit 1
[ -f mmla_audio_amd/ab/libmmla_rawstage.so ] && { bash tools/gpu/ab.sh od_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_rawstage.so 2 || exit 1; }
[ -n "$SIPMC" ] && { bash tools/gpu/pmc_kernels.sh si_pipeline 16384 r4si > gpurun_out/pmc_r4si.log 2>&1 || { tail -20 gpurun_out/pmc_r4si.log; exit 1; }; head -30 gpurun_out/pmc_r4si_summary.txt; }
exit 0
