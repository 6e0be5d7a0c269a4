#!/bin/bash
# HBM traffic of the roofline kernels from PMC (separate FETCH_SIZE / WRITE_SIZE passes, as the
# MI355X guide prescribes), written to gpurun_out/pmc_traffic_<workload>.json for profiles/.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in ${PMC_WL:-od_pipeline od_features si_pipeline}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmct_${wl}_$ctr
    timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmct_${wl}_$ctr -o p -- python3 -u bench.py --workload $wl --steps 1 --warmup 0 --no-cpu-baseline --no-f32 --no-parity --no-latency > gpurun_out/pmct_${wl}_$ctr.log 2>&1 || exit $?
  done
  python3 tools/pmc_traffic.py $wl gpurun_out/pmct_${wl}_FETCH_SIZE gpurun_out/pmct_${wl}_WRITE_SIZE gpurun_out/pmct_${wl}_FETCH_SIZE.log > gpurun_out/pmc_traffic_$wl.json || exit $?
  cat gpurun_out/pmc_traffic_$wl.json
  rm -rf gpurun_out/pmct_${wl}_*
done
