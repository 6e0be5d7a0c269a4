#!/bin/bash
# variant check: parity sample of a variant build on a workload, then A/B against the product build
#   var_check.sh <variant.so> <workload> [rounds]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$1; wl=$2; r=${3:-2}
timeout -k 10 300 python3 tools/bench_with_lib.py $V --workload $wl --no-cpu-baseline --no-f32 --no-latency --steps 1 --warmup 1 > gpurun_out/vc.log 2>&1 || { tail -20 gpurun_out/vc.log; exit 1; }
grep '^{' gpurun_out/vc.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$(basename $V) parity', {k: v for k, v in d['parity'].items() if k != 'sample'})"
bash tools/gpu/ab.sh $wl mmla_audio_amd/libmmla.so $V $r
