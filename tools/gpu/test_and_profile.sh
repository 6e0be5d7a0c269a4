#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_tp.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_tp.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/pytest_tp.log | head; exit $rc; fi
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tp -o od -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_tp.log 2>&1 || exit $?
tail -1 gpurun_out/prof_tp.log | cut -c 1-200
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_tp/od_kernel_stats.csv')))
mine=[r for r in rows if 'anonymous' in r['Name']]
tot=sum(int(r['TotalDurationNs']) for r in mine)
print('total ms', tot/1e6)
for r in mine[:16]: print(f"{r['Name'][:80]:80s} {r['Calls']:>5} avg {float(r['AverageNs'])/1e6:8.3f} ms {100*int(r['TotalDurationNs'])/tot:5.1f}%")
PY
# keep only the stats summaries (traces exceed gpurun's copy-back limit)
find gpurun_out/prof_tp -type f ! -name '*_stats.csv' -delete
