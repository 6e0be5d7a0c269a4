cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "si" --timeout 200 --timeout-method thread > gpurun_out/sq.log 2>&1; rc=$?; tail -2 gpurun_out/sq.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python3 tools/lib_probs.py mmla_audio_amd/ab/libmmla_head.so gpurun_out/p_head.npy si 8192 > gpurun_out/lp.log 2>&1 || { tail gpurun_out/lp.log; exit 1; }
timeout -k 10 200 python3 tools/lib_probs.py mmla_audio_amd/libmmla.so gpurun_out/p_new.npy si 8192 >> gpurun_out/lp.log 2>&1 || { tail gpurun_out/lp.log; exit 1; }
cmp gpurun_out/p_head.npy gpurun_out/p_new.npy && echo BIT-IDENTICAL
rm -f gpurun_out/p_*.npy
bash tools/gpu/ab.sh si_pipeline mmla_audio_amd/ab/libmmla_head.so mmla_audio_amd/libmmla.so 2
