#!/bin/bash
# resblk block-1 phase timeline (RB_EXP=4 build)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
MMLA_LIB=mmla_audio_amd/ab/libmmla_e4.so timeout -k 10 300 python3 tools/rb_timeline.py 2>&1 | grep -v amdgpu.ids
