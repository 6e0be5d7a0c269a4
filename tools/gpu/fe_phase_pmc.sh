#!/bin/bash
# SQ instruction counts of the OD front-end per phase-skip build (FE3_SKIP, see fe_phase_skip.sh):
# the difference to the full build is the phase's instruction count
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${SKIPS:-0 1 2 4 8 16}; do
  if [ $v = 0 ]; then lib=mmla_audio_amd/libmmla.so; else lib=mmla_audio_amd/ab/libmmla_skip$v.so; fi
  rm -rf gpurun_out/fpmc_$v
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/fpmc_$v -o p -- python3 tools/bench_with_lib.py $lib --workload od_features --clips 4096 --steps 1 --warmup 0 --no-cpu-baseline --no-f32 --no-parity --no-latency > gpurun_out/fpmc_$v.log 2>&1 || { echo "pass $v failed"; tail -5 gpurun_out/fpmc_$v.log; exit 1; }
  python3 - $v <<'PY'
import csv, glob, sys, collections
v = sys.argv[1]
f = glob.glob(f'gpurun_out/fpmc_{v}/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(float); n = 0
for r in csv.DictReader(open(f)):
    if 'od_fe3' not in r['Kernel_Name']: continue
    acc[r['Counter_Name']] += float(r['Counter_Value'])
disp = len({r['Dispatch_Id'] for r in csv.DictReader(open(f)) if 'od_fe3' in r['Kernel_Name']})
print('skip', v, 'dispatches', disp, ' '.join(f"{k}={acc[k]/disp/4096:.0f}/clip" for k in sorted(acc)))
PY
  rm -rf gpurun_out/fpmc_$v
done
