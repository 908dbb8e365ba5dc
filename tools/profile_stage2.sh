#!/bin/bash
# rocprofv3 kernel trace of bench_stage2.py (Stage II at the config-2 shape): the per-kernel
# summary, plus per-dispatch durations of the LU kernels of the last factorization.
set -euo pipefail
export TMPDIR=/tmp
raw=$(mktemp -d /tmp/ps2_XXXX)
mkdir -p gpurun_out/prof_stage2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$raw" -o run -- \
  python3 bench_stage2.py --cpu-sample 0 > gpurun_out/prof_stage2/log.txt 2>&1
cp "$(find "$raw" -name "*kernel_stats.csv" | head -1)" gpurun_out/prof_stage2/r01_stage2_kernel_stats.csv
python3 - "$(find "$raw" -name "*kernel_trace.csv" | head -1)" > gpurun_out/prof_stage2/lu_dispatches.txt <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "iadmm::lu_" in r["Kernel_Name"] and "solve" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
per = len(rows) // 4  # warmup, 2 steps, 1 standalone factor
for r in rows[-per:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f'{r["Kernel_Name"][:40]:40s} grid={r.get("Grid_Size_X", r.get("Grid_Size", "?"))}x{r.get("Grid_Size_Y", "")} us={d:9.1f}')
PY
rm -rf "$raw"
