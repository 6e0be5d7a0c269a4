#!/bin/bash
# rocprofv3 kernel-trace stats of one bench line: WL=<workload> TAG=<name>
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
wl=${WL:-od_pipeline}; tag=${TAG:-$wl}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --workload $wl --no-cpu-baseline --no-f32 --no-parity ${BENCH_ARGS} > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
f=$(find gpurun_out/prof_$tag -name '*kernel_stats.csv' | head -1)
cp $f gpurun_out/${tag}_kernel_stats.csv
rm -rf gpurun_out/prof_$tag   # traces exceed gpurun's copy-back limit
python3 - <<PY
import csv
rows=list(csv.DictReader(open('gpurun_out/${tag}_kernel_stats.csv')))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:25]:
    print('%6.2f%% %8d %10.3f ms avg %8.3f ms  %s'%(100*float(r['TotalDurationNs'])/tot,int(r['Calls']),float(r['TotalDurationNs'])/1e6,float(r['AverageNs'])/1e6,r['Name'][:150]))
PY
grep '^{' gpurun_out/prof_$tag.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['roofline']['avg_launch_ms'])"
