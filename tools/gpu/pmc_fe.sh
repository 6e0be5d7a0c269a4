#!/bin/bash
# PMC passes (issue/stall picture) over the OD pipeline bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_BRANCH" "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQ_IFETCH_LEVEL" "SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_TRANS_F"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc13_$i
  timeout -k 10 600 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc13_$i -o p -- python3 bench.py --workload od_features --clips 16384 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc13_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc13_$i.log; }
done
python3 tools/pmc_summary.py gpurun_out/pmc13_* --match od_fe > gpurun_out/pmc13_summary.txt
rm -rf gpurun_out/pmc13_[0-9]*
cat gpurun_out/pmc13_summary.txt
