#!/bin/bash
# OD front-end: parity tests, throughput vs batch size, phase timeline; SI pipeline kernel profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "od_features" --timeout 120 --timeout-method thread > gpurun_out/od_fe_tests.log 2>&1
rc=$?; tail -3 gpurun_out/od_fe_tests.log; [ $rc -eq 0 ] || exit $rc
for n in 4096 65536; do
  timeout -k 10 300 python3 bench.py --workload od_features --clips $n --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fe_$n.log 2>&1 || exit $?
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/fe_$n.log') if l.startswith('{')][0]);r=d['roofline'];print($n,'clips/s',round(d['value']),'launch ms',round(r['avg_launch_ms'],4),'frac',round(r['frac'],4))"
done
timeout -k 10 300 python3 tools/fe_timeline.py > gpurun_out/fe_timeline.log 2>&1 || exit $?
cat gpurun_out/fe_timeline.log | grep -v amdgpu.ids
exit 0
rm -rf gpurun_out/prof_si
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_si -o si -- python3 bench.py --workload si_pipeline --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_si.log 2>&1 || exit $?
find gpurun_out/prof_si -type f ! -name '*_stats.csv' -delete
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/prof_si/**/si_kernel_stats.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(int(r['TotalDurationNs']) for r in rows)
for r in rows[:14]: print(f"{r['Name'][:90]:90s} {r['Calls']:>5} avg {float(r['AverageNs'])/1e6:8.3f} ms {100*int(r['TotalDurationNs'])/tot:5.1f}%")
PY
