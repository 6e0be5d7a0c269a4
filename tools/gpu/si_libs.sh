#!/bin/bash
# kernel stats of the SI conv stack for several library builds: si_libs.sh lib1.so lib2.so ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for L in "$@"; do
  rm -rf gpurun_out/ks_s
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_s -o run -- python3 tools/bench_with_lib.py $L --workload si_pipeline --steps 3 --warmup 1 --no-cpu-baseline --no-latency --no-f32 > gpurun_out/ks_s.json 2> gpurun_out/ks_s.log || { echo "kstats rc=$?"; tail -5 gpurun_out/ks_s.log; exit 1; }
  f=$(find gpurun_out/ks_s -name "*kernel_stats.csv" | head -1)
  echo "== $L"
  python3 - "$f" <<'PY'
import csv, sys, json
tot = 0.0
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    if any(k in n for k in ('siu', 'conv_h3', 'si_fe', 'bilstm')):
        print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e6:9.3f} ms  {n[:90]}")
        if 'siu' in n:
            tot += float(r['TotalDurationNs']) / 1e6
d = json.loads([l for l in open('gpurun_out/ks_s.json') if l.startswith('{')][0])
print('siu total ms', round(tot, 3), 'value', round(d['value']), 'roof', d['roofline']['kernel'], round(d['roofline']['frac'], 4), 'conv frac', round((d.get('roofline_conv') or d['roofline'])['frac'], 4),
      'parity', d['parity'])
PY
done
rm -rf gpurun_out/ks_s
