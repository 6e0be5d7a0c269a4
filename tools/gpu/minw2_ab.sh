#!/bin/bash
# conv_h3 register budgets re-measured after the fragment-order weights
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu/ab.sh si_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_si2.so 2 || exit 1
bash tools/gpu/ab.sh od_pipeline mmla_audio_amd/libmmla.so mmla_audio_amd/ab/libmmla_r2.so 2
