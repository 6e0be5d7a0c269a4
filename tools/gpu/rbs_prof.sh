#!/bin/bash
# kernel stats of the OD pipeline with tiles (MMLA_RB_TILE=1) and strips, then SQ/TCP counters of the strips
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in 1 0; do
  rm -rf gpurun_out/ks_$t
  MMLA_RB_TILE=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_$t -o run -- python3 bench.py --clips 16384 --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-f32 --no-parity > gpurun_out/ks_$t.log 2>&1 || { echo "kstats rc=$?"; tail -5 gpurun_out/ks_$t.log; exit 1; }
  f=$(find gpurun_out/ks_$t -name "*kernel_stats.csv" | head -1)
  echo "== tile=$t"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    if any(k in n for k in ('odu', 'resblk', 'rbs')):
        print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e6:9.3f} ms  {n[:110]}")
PY
  rm -f gpurun_out/ks_$t/*/*kernel_trace.csv gpurun_out/ks_$t/*kernel_trace.csv
done
i=0
for set in "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_rbs_$i
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_rbs_$i -o p -- python3 bench.py --clips 4096 --steps 1 --warmup 0 --no-cpu-baseline --no-f32 --no-parity --no-latency > gpurun_out/pmc_rbs_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_rbs_$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc_rbs_[0-9]* > gpurun_out/pmc_rbs_summary.txt
rm -rf gpurun_out/pmc_rbs_[0-9]*
grep -A12 -i "rbs\|resblk" gpurun_out/pmc_rbs_summary.txt | head -60
