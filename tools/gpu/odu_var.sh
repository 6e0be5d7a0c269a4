#!/bin/bash
# dev (round 5): odu tile-geometry variants (env MMLA_ODU_VARIANT) -> per-kernel rocprof averages
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  d=gpurun_out/odu_var$v
  mkdir -p $d
  MMLA_ODU_VARIANT=$v timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --no-cpu-baseline --no-latency --no-f32 --no-parity > $d/bench.json 2> $d/bench.err || { echo "rc=$?"; tail -20 $d/bench.err; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print('variant', sys.argv[2])
for r in rows:
    n = r['Name']
    if any(k in n for k in ('odu', 'resblk', 'conv_h3')):
        print(f"  {int(r['Calls']):5d} {float(r['AverageNs'])/1e6:9.3f} ms  {n[:110]}")
PY
  rm -f $d/*kernel_trace.csv $d/*.db
done
