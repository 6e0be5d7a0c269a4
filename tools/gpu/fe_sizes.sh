#!/bin/bash
# front-end line at config 2 (4096 clips) and at 65 536 clips: v3 (the product library) and, when an
# A/B build mmla_audio_amd/ab/libmmla_v2.so (-DOD_FE_V2_AB=1) is present, v2 (MMLA_OD_FE_V2=1)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
libs="mmla_audio_amd/libmmla.so"
[ -f mmla_audio_amd/ab/libmmla_v2.so ] && libs="$libs mmla_audio_amd/ab/libmmla_v2.so"
for n in 4096 65536; do
  for lib in $libs; do
    case $lib in *v2*) v=1;; *) v=0;; esac
    MMLA_OD_FE_V2=$v timeout -k 10 300 python3 tools/bench_with_lib.py $lib --workload od_features --clips $n --no-cpu-baseline --no-parity --no-latency --steps 50 > gpurun_out/fes.log 2>&1 || { tail -20 gpurun_out/fes.log; exit 1; }
    grep '^{' gpurun_out/fes.log | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('clips $n v2=$v', round(d['value']), round(r['avg_launch_ms'],4), round(r['frac'],4))"
  done
done
