#!/bin/bash
# r05: kernel traces of one factorization (B = 1024, N = 2000), paired (third form) vs rank-128, one stream and look-ahead
# stream (no look-ahead: clean per-kernel durations) and paired with the look-ahead
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05k
for cfg in "pair1 2 --no-lookahead" "pairla 2" "r128la 0"; do
  set -- $cfg
  raw=$(mktemp -d /tmp/lu_XXXX)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$raw" -o run -- python3 tools/profile_lu.py --flags $2 $3 \
    > gpurun_out/r05k/$1.log 2>&1 || exit $?
  cp "$(find "$raw" -name "*kernel_stats.csv" | head -1)" gpurun_out/r05k/$1_kernel_stats.csv
  python3 -c "import csv,sys; r=csv.DictReader(open(sys.argv[1])); w=None
for row in r:
    if 'iadmm' not in row['Kernel_Name']: continue
    if w is None: w=csv.DictWriter(open(sys.argv[2],'w'), fieldnames=['Kernel_Name','Start_Timestamp','End_Timestamp','Stream_Id']); w.writeheader()
    w.writerow({k: row.get(k, '') for k in ['Kernel_Name','Start_Timestamp','End_Timestamp','Stream_Id']})" \
    "$(find "$raw" -name "*kernel_trace.csv" | head -1)" gpurun_out/r05k/$1_kernel_trace.csv
  rm -rf "$raw"
done
echo done
