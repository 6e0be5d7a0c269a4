#!/bin/bash
# dev: rocprof kernel stats of the OD pipeline bench (3xFP16 path only) -> gpurun_out/prof_od/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_od
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_od -o run -- python3 bench.py --no-cpu-baseline --no-latency --no-f32 --no-parity > gpurun_out/prof_od/bench.json 2> gpurun_out/prof_od/bench.err || { echo "rc=$?"; tail -20 gpurun_out/prof_od/bench.err; exit 1; }
f=$(find gpurun_out/prof_od -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/prof_od/kernel_stats.csv
rm -f gpurun_out/prof_od/*kernel_trace.csv gpurun_out/prof_od/*.db
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/prof_od/kernel_stats.csv')))
for r in rows:
    n = r['Name']
    if any(k in n for k in ('odu', 'resblk', 'conv_h3', 'od_fe3', 'bilstm', 'mean_h', 'od_head')):
        print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e6:9.3f} ms  {n[:150]}")
PY
