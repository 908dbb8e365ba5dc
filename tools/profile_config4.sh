#!/bin/bash
# BASELINE config 4 on one MI355X (n=5000, m=2500+2500, h=2048, B=512, K=200), run from the repo
# root on the GPU box:
#   1. FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes over a 2-iteration solve of
#      the same instances (per-launch counters do not depend on K), summarised per kernel into
#      profiles/<tag>_pmc_<ctr>_n5000_m5000_h2048_B512.csv (bench.py reads them for "traffic");
#   2. the full K=200 bench step (in-place scaling: Q, A0 and their scaled copies would need
#      204 GB next to 126 GB of H/C);
#   3. Stage II at the config-4 shape (N = 10000: 8-column LU panels, batch-chunked K).
# Results land in gpurun_out/<tag>_cfg4/ (copy them into profiles/).
# Usage: bash tools/profile_config4.sh <tag>
set -euo pipefail
tag=${1:-r02}
out=gpurun_out/${tag}_cfg4
mkdir -p "$out" profiles
export TMPDIR=/tmp
raw=$(mktemp -d /tmp/cfg4_XXXX)
C4="--batch 512 --num_var 5000 --num_ineq 2500 --num_eq 2500 --hidden_dim 2048"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 600 rocprofv3 --pmc $ctr --output-format csv -d "$raw/pmc_$ctr" -o run -- \
    python3 bench.py $C4 --outer_T 2 --steps 1 --warmup 0 --cpu-sample 0 --alt-f16x3 0 --train-batch 0 --stage2-iters 0 --in-place-scaling \
    > "$out/pmc_$ctr.log" 2>&1
  python3 tools/pmc_summary.py "$(find "$raw/pmc_$ctr" -name "*counter_collection.csv" | head -1)" \
    > "profiles/${tag}_pmc_${ctr}_n5000_m5000_h2048_B512.csv"
  cp "profiles/${tag}_pmc_${ctr}_n5000_m5000_h2048_B512.csv" "$out/"
  rm -rf "$raw/pmc_$ctr"
done
rm -rf "$raw"
timeout -k 10 700 python3 -u bench.py $C4 --outer_T 200 --steps 1 --warmup 0 --cpu-sample 0 --alt-f16x3 0 --train-batch 0 --stage2-iters 0 \
  --in-place-scaling > "$out/bench_config4.json" 2> "$out/bench_config4.err"
[ "${SKIP_STAGE2:-0}" = 1 ] || timeout -k 10 400 python3 -u bench_stage2.py --batch 512 --num_var 5000 --num_ineq 2500 --num_eq 2500 \
  --steps 1 --warmup 0 --cpu-sample 0 > "$out/stage2_config4.json" 2> "$out/stage2_config4.err"
echo "config-4 profile done: $out"
