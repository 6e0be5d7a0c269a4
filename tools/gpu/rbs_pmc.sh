#!/bin/bash
# SQ counters of the strip kernels (one library): rbs_pmc.sh [lib.so]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=${1:-mmla_audio_amd/libmmla.so}
i=0
for set in "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH" "SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR" "SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_MFMA SQ_INSTS_SMEM SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_rbs_$i
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_rbs_$i -o p -- python3 tools/bench_with_lib.py $L --clips 4096 --steps 1 --warmup 0 --no-cpu-baseline --no-f32 --no-parity --no-latency > gpurun_out/pmc_rbs_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_rbs_$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_rbs_[0-9]* > gpurun_out/pmc_rbs_summary.txt
rm -rf gpurun_out/pmc_rbs_[0-9]*
grep -A3 "rbs_kernel" gpurun_out/pmc_rbs_summary.txt
