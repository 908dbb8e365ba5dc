#!/bin/bash
# Stage-II LU factorization profile on the GPU box: kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes, each over ONE factorization (tools/profile_lu.py), summarised
# into gpurun_out/prof_lu_<tag>/<tag>_stage2_{kernel_stats,pmc_*}_N<N>_B<B>.csv (copy them into
# profiles/: bench.py's stage2 roofline reads the PMC pair).  Usage: bash tools/profile_lu.sh <tag> [B] [N]
set -euo pipefail
tag=${1:-r03}; B=${2:-1024}; N=${3:-2000}
export TMPDIR=/tmp
raw=$(mktemp -d /tmp/lu_XXXX)
out=gpurun_out/prof_lu_$tag
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$raw/trace" -o run -- python3 tools/profile_lu.py --batch $B --N $N \
  > "$out/trace.log" 2>&1
cp "$(find "$raw/trace" -name "*kernel_stats.csv" | head -1)" "$out/${tag}_stage2_kernel_stats_N${N}_B${B}.csv"
cp "$(find "$raw/trace" -name "*kernel_trace.csv" | head -1)" "$out/${tag}_stage2_kernel_trace_N${N}_B${B}.csv"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d "$raw/pmc_$ctr" -o run -- \
    python3 tools/profile_lu.py --batch $B --N $N > "$out/pmc_$ctr.log" 2>&1
  python3 tools/pmc_summary.py "$(find "$raw/pmc_$ctr" -name "*counter_collection.csv" | head -1)" \
    > "$out/${tag}_stage2_pmc_${ctr}_N${N}_B${B}.csv"
done
rm -rf "$raw"
echo "LU profile done"
