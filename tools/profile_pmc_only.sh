#!/bin/bash
set -euo pipefail
export TMPDIR=/tmp
sum=gpurun_out/prof_r01/summary
mkdir -p $sum
raw=$(mktemp -d /tmp/prof_XXXX)
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --pmc $ctr --output-format csv -d "$raw/pmc_$ctr" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --alt-f16x3 0 > "$sum/bench_pmc_$ctr.log" 2>&1
  python3 tools/pmc_summary.py "$(find "$raw/pmc_$ctr" -name "*counter_collection.csv" | head -1)" \
    > "$sum/r01_pmc_${ctr}_n1000_m1000_h800_B1024.csv"
done
rm -rf "$raw"
