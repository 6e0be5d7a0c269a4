#!/bin/bash
# per-kernel rocprof of two library builds: prof_ab.sh <workload> <libA.so> <libB.so>
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
wl=$1
i=0
for L in $2 $3; do
  i=$((i+1))
  rm -rf gpurun_out/pab_$i
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/pab_$i -o run -- python3 tools/bench_with_lib.py $L --workload $wl --no-cpu-baseline --no-f32 --no-parity --steps 1 > gpurun_out/pab_$i.log 2>&1 || { tail -20 gpurun_out/pab_$i.log; exit 1; }
  db=$(find gpurun_out/pab_$i -name '*.db' | head -1)
  echo "== $L"; python3 tools/prof_db.py $db | grep -v "^ *0\.[0-4]%"
  python3 tools/prof_db.py $db --csv gpurun_out/pab_$i.csv > /dev/null
  rm -rf gpurun_out/pab_$i   # the database is tens of MB; the CSV summary stays
done
