#!/bin/bash
# rocprofv3 evidence for the bench line (run on the GPU box from the repo root):
#   1. kernel trace + stats of one bench step (per-kernel average durations),
#   2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes (TCC block limits), summarised per kernel
#      by tools/pmc_summary.py.
# Summaries land in gpurun_out/prof_<tag>/summary/ (copy them into profiles/); the raw traces are
# deleted at the end (they exceed what gpurun copies back).
# (--train-batch 0 --stage2-iters 0: the headline solve only; r03: a --pmc pass through the training
# record segfaulted inside the profiler's dispatch interception, rc 139)
# Usage: bash tools/profile_bench.sh <tag>     (e.g. r01)
set -euo pipefail
tag=${1:-r01}
out=gpurun_out/prof_$tag
sum=$out/summary
mkdir -p "$out" "$sum"
export TMPDIR=/tmp
raw=$(mktemp -d /tmp/prof_XXXX)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$raw/trace" -o run -- \
  python3 bench.py --steps 1 --warmup 1 --cpu-sample 0 --alt-f16x3 0 --train-batch 0 --stage2-iters 0 > "$sum/bench_trace.log" 2>&1
cp "$(find "$raw/trace" -name "*kernel_stats.csv" | head -1)" "$sum/${tag}_bench_kernel_stats.csv"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --pmc $ctr --output-format csv -d "$raw/pmc_$ctr" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 --alt-f16x3 0 --train-batch 0 --stage2-iters 0 > "$sum/bench_pmc_$ctr.log" 2>&1
  python3 tools/pmc_summary.py "$(find "$raw/pmc_$ctr" -name "*counter_collection.csv" | head -1)" \
    > "$sum/${tag}_pmc_${ctr}_n1000_m1000_h800_B1024.csv"
done
rm -rf "$raw"
grep -h '^{' "$sum/bench_trace.log" > "$sum/${tag}_bench_under_trace.json" || true
echo "profile done: $sum"
