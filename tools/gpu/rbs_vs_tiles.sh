#!/bin/bash
# blocks 1-3: rolling strips (default) against the round-5 16x16 tiles (MMLA_RB_TILE=1), same box, twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for mode in strips tiles strips tiles; do
  rm -rf gpurun_out/ks_t
  if [ $mode = tiles ]; then export MMLA_RB_TILE=1; else unset MMLA_RB_TILE; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_t -o run -- python3 bench.py --clips 16384 --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-f32 --no-parity > gpurun_out/ks_t.json 2> gpurun_out/ks_t.log || { echo "rc=$?"; tail -5 gpurun_out/ks_t.log; exit 1; }
  f=$(find gpurun_out/ks_t -name "*kernel_stats.csv" | head -1)
  echo "== $mode"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r['Name'] for k in ('resblk_kernel', 'rbs_kernel', 'odu_kernel<64, 76')):
        print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e6:9.3f} ms  {r['Name'][:90]}")
PY
done
unset MMLA_RB_TILE
rm -rf gpurun_out/ks_t
