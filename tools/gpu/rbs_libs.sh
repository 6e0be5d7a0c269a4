#!/bin/bash
# kernel stats of the blocks 1-3 strips for several library builds: rbs_libs.sh lib1.so lib2.so ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for L in "$@"; do
  rm -rf gpurun_out/ks_l
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_l -o run -- python3 tools/bench_with_lib.py $L --clips 16384 --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-f32 > gpurun_out/ks_l.json 2> gpurun_out/ks_l.log || { echo "kstats rc=$?"; tail -5 gpurun_out/ks_l.log; exit 1; }
  f=$(find gpurun_out/ks_l -name "*kernel_stats.csv" | head -1)
  echo "== $L"
  python3 - "$f" <<'PY'
import csv, sys, json
tot = 0.0
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    if any(k in n for k in ('odu', 'resblk', 'rbs')):
        print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e6:9.3f} ms  {n[:100]}")
d = json.loads([l for l in open('gpurun_out/ks_l.json') if l.startswith('{')][0])
print('value', round(d['value']), 'conv frac', round(d['roofline']['frac'], 4), 'logp_net', d['parity']['logp_err_net'])
PY
done
rm -rf gpurun_out/ks_l
