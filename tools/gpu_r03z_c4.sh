#!/bin/bash
# Config-4 Stage II: balanced chunks (default) against the r03 first-session split (--chunk 410).
set -o pipefail
mkdir -p gpurun_out/r03z7
for c in 0 410; do
  timeout -k 10 500 python3 -u bench_stage2.py --batch 512 --num_var 5000 --num_ineq 2500 --num_eq 2500 \
    --steps 1 --warmup 0 --cpu-sample 0 --chunk $c > gpurun_out/r03z7/stage2_config4_chunk$c.json 2> gpurun_out/r03z7/stage2_config4_chunk$c.err || exit 1
  grep '^{' gpurun_out/r03z7/stage2_config4_chunk$c.json | cut -c1-400
done
