#!/bin/bash
# Round-2 issue/stall picture (SQ counters, one pass per set) of the FE, SI and OD bench lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # workload clips tag
  local wl=$1 n=$2 tag=$3 i=0
  for set in "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_BRANCH" "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM"; do
    i=$((i+1))
    rm -rf gpurun_out/pmc_${tag}_$i
    timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_${tag}_$i -o p -- python3 bench.py --workload $wl --clips $n --steps 1 --warmup 0 --no-cpu-baseline --no-f32 --no-parity --no-latency > gpurun_out/pmc_${tag}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_${tag}_$i.log; return 1; }
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_${tag}_[0-9]* > gpurun_out/r2_pmc_${tag}_summary.txt
  rm -rf gpurun_out/pmc_${tag}_[0-9]*
  cat gpurun_out/r2_pmc_${tag}_summary.txt
}


run od_pipeline 16384 od_pipeline || exit 1
