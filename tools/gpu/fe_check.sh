#!/bin/bash
# front-end change check: GPU suite, A/B against a reference build ($1), SQ instruction counts of the
# current build's od_fe3 kernel (config 2, 4096 clips)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fc_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/fc_pytest.log; [ $rc = 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/fc_pytest.log | head; exit 1; }
bash tools/gpu/fe_ab.sh ${1:-mmla_audio_amd/ab/libmmla_head.so} mmla_audio_amd/libmmla.so 2 || exit 1
rm -rf gpurun_out/fcpmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/fcpmc -o p -- python3 bench.py --workload od_features --clips 4096 --steps 1 --warmup 0 --no-cpu-baseline --no-f32 --no-parity --no-latency > gpurun_out/fcpmc.log 2>&1 || { tail -5 gpurun_out/fcpmc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/fcpmc/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    if 'od_fe3' in r['Kernel_Name']: acc[r['Counter_Name']] += float(r['Counter_Value'])
print(' '.join(f"{k}={acc[k]/4096:.0f}/clip" for k in sorted(acc)))
PY
rm -rf gpurun_out/fcpmc
