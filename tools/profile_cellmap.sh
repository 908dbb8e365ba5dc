#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the cell kernel per tile order (tools/cellmap.py, one group size per
# rocprofv3 --pmc pass).  Summaries: gpurun_out/prof_cellmap/<ctr>_pg<g>.csv
# Usage: bash tools/profile_cellmap.sh "1 4 8"
set -euo pipefail
export TMPDIR=/tmp
out=gpurun_out/prof_cellmap
mkdir -p "$out"
raw=$(mktemp -d /tmp/prof_XXXX)
for pg in ${1:-1 4}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$raw/${ctr}_$pg" -o run -- \
      python3 tools/cellmap.py --groups $pg --reps 1 > "$out/${ctr}_pg$pg.log" 2>&1
    python3 tools/pmc_summary.py "$(find "$raw/${ctr}_$pg" -name "*counter_collection.csv" | head -1)" \
      > "$out/${ctr}_pg$pg.csv"
  done
done
rm -rf "$raw"
echo "done: $out"
