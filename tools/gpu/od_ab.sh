#!/bin/bash
# dev: OD bit-identity of the current build against a reference build ($1), then alternating A/B
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
REF=${1:-mmla_audio_amd/ab/libmmla_head.so}
timeout -k 10 200 python3 tools/lib_probs.py $REF gpurun_out/p_ref.npy od 4096 > gpurun_out/lp.log 2>&1 || { tail gpurun_out/lp.log; exit 1; }
timeout -k 10 200 python3 tools/lib_probs.py mmla_audio_amd/libmmla.so gpurun_out/p_new.npy od 4096 >> gpurun_out/lp.log 2>&1 || { tail gpurun_out/lp.log; exit 1; }
cmp gpurun_out/p_ref.npy gpurun_out/p_new.npy && echo BIT-IDENTICAL
rm -f gpurun_out/p_*.npy
bash tools/gpu/ab.sh od_pipeline $REF mmla_audio_amd/libmmla.so ${2:-2}
