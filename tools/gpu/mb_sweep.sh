#!/bin/bash
# micro-batch sweep: bash tools/gpu/mb_sweep.sh <workload> <mb> [<mb> ...]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
wl=$1; shift
for mb in "$@"; do
  timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline --microbatch $mb > gpurun_out/mb_${wl}_$mb.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/mb_${wl}_$mb.log') if l.startswith('{')][-1]); print('$wl mb $mb', round(d['value']), round(d['ms_per_step'],2))"
done
