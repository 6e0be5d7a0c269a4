#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu/test_and_profile.sh || exit $?
cp mmla_audio_amd/libmmla_e4.so mmla_audio_amd/libmmla.so
timeout -k 10 300 python3 tools/rb_timeline.py
