#!/bin/bash
# rbs dev loop: its tests, then kernel stats of the strips (tiles: resblk<16,32> 23.15 ms, <32,32> 9.56 ms per 16 384 clips)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rbs.py > gpurun_out/rbs_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/rbs_tests.log; exit 1; }
tail -2 gpurun_out/rbs_tests.log
rm -rf gpurun_out/ks_q
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_q -o run -- python3 bench.py --clips 16384 --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-f32 > gpurun_out/ks_q.json 2> gpurun_out/ks_q.log || { echo "kstats rc=$?"; tail -5 gpurun_out/ks_q.log; exit 1; }
f=$(find gpurun_out/ks_q -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, json
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    if any(k in n for k in ('odu', 'resblk', 'rbs')):
        print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e6:9.3f} ms  {n[:100]}")
d = json.loads(open('gpurun_out/ks_q.json').read())
print('value', round(d['value']), 'conv frac', round(d['roofline']['frac'], 4), 'logp_net', d['parity']['logp_err_net'])
PY
rm -rf gpurun_out/ks_q
