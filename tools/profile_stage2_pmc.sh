#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the Stage-II kernels (one --pmc pass per counter, own run each),
# bench_stage2.py at the config-2 shape, one step.  Summaries: gpurun_out/prof_stage2_pmc/.
set -euo pipefail
export TMPDIR=/tmp
sum=gpurun_out/prof_stage2_pmc
mkdir -p $sum
raw=$(mktemp -d /tmp/ps2pmc_XXXX)
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --pmc $ctr --output-format csv -d "$raw/pmc_$ctr" -o run -- \
    python3 bench_stage2.py --steps 1 --warmup 0 --cpu-sample 0 --iters 2 > "$sum/pmc_$ctr.log" 2>&1
  python3 tools/pmc_summary.py "$(find "$raw/pmc_$ctr" -name "*counter_collection.csv" | head -1)" \
    > "$sum/r01_stage2_pmc_${ctr}_N2000_B1024.csv"
done
rm -rf "$raw"
