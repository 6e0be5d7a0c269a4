#!/bin/bash
# rocprof kernel stats of the SI pipeline bench (our kernels only)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_si
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_si -o si -- python3 -u bench.py --workload si_pipeline --steps 2 --warmup 1 --no-cpu-baseline --no-f32 --no-parity --no-latency > gpurun_out/prof_si.log 2>&1 || exit $?
find gpurun_out/prof_si -type f ! -name '*_stats.csv' -delete
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_si/**/si_kernel_stats.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if 'at::native' not in r['Name']]
tot = sum(int(r['TotalDurationNs']) for r in rows)
print('total ms', tot / 1e6)
for r in rows: print(f"{r['Name'][:95]:95s} {r['Calls']:>5} avg {float(r['AverageNs'])/1e6:8.3f} ms {100*int(r['TotalDurationNs'])/tot:5.1f}%")
PY
