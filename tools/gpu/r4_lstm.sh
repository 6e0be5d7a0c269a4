#!/bin/bash
# round 4: VALU rate probe; bit-identity of the fused SI pool units (MMLA_NO_SIPU) and of the
# LSTM_W4 variant (OD + SI probabilities); the SI fused-unit / batching / parity tests; A/Bs; then the
# whole GPU suite.  Each GPU step under its own time limit; stops at the first failure.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
P=mmla_audio_amd/libmmla.so
V=mmla_audio_amd/ab/libmmla_lstmw4.so
timeout -k 10 60 ./tools/ubench/valu_rates 2100 > gpurun_out/valu_rates.txt 2>&1 || exit 1
cat gpurun_out/valu_rates.txt
lp() { timeout -k 10 200 python3 tools/lib_probs.py "$@" > gpurun_out/lp.log 2>&1 || { tail -20 gpurun_out/lp.log; exit 1; }; }
export MMLA_NO_SIPU=0 MMLA_NO_SIFIN=0
lp $P gpurun_out/p_si.npy si
MMLA_NO_SIPU=1 lp $P gpurun_out/q_si.npy si
cmp gpurun_out/p_si.npy gpurun_out/q_si.npy && echo "sipu: si bit-identical" || echo "sipu: si DIFFERS"
MMLA_NO_SIFIN=1 lp $P gpurun_out/f_si.npy si
cmp gpurun_out/p_si.npy gpurun_out/f_si.npy && echo "sifin: si bit-identical" || echo "sifin: si DIFFERS"
lp $V gpurun_out/v_si.npy si
cmp gpurun_out/p_si.npy gpurun_out/v_si.npy && echo "lstm_w4: si bit-identical" || echo "lstm_w4: si DIFFERS"
lp $P gpurun_out/p_od.npy od
lp $V gpurun_out/v_od.npy od
cmp gpurun_out/p_od.npy gpurun_out/v_od.npy && echo "lstm_w4: od bit-identical" || echo "lstm_w4: od DIFFERS"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_siu.py tests/test_gpu_batching.py tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread > gpurun_out/r4_first.log 2>&1
rc=$?; tail -3 gpurun_out/r4_first.log; [ $rc = 0 ] || exit 1
unset MMLA_NO_SIPU MMLA_NO_SIFIN
bash tools/gpu/env_ab.sh si_pipeline "MMLA_NO_SIPU=1 MMLA_NO_SIFIN=1" "MMLA_NO_SIPU=0 MMLA_NO_SIFIN=1" 2 || exit 1
bash tools/gpu/env_ab.sh si_pipeline "MMLA_NO_SIPU=0 MMLA_NO_SIFIN=1" "MMLA_NO_SIPU=0 MMLA_NO_SIFIN=0" 2 || exit 1
export MMLA_NO_SIPU=0 MMLA_NO_SIFIN=0
bash tools/gpu/abn.sh si_pipeline 2 $P $V mmla_audio_amd/ab/libmmla_lstmw4p.so || exit 1
bash tools/gpu/abn.sh od_pipeline 1 $P $V mmla_audio_amd/ab/libmmla_lstmw4p.so || exit 1
NOSUITE=${NOSUITE:-} bash tools/gpu/r4_check.sh
