#!/bin/bash
# r03: LU tests, A/B timing and per-kernel stats of one factorization (B = 1024, N = 2000) for the
# default build and variants/*.so
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03c
bash tools/gpu_tests.sh r03c 600 tests/test_stage2_gpu.py || exit 1
timeout -k 10 400 python3 -u tools/lu_ab.py --libs i-admm-lstm_amd/iadmm/libiadmm.so variants/*.so \
  --batch 1024 --N 2000 > gpurun_out/r03c/lu_ab.txt 2>&1 || exit 1
grep '^{' gpurun_out/r03c/lu_ab.txt | cut -c1-220
for v in default variants/*.so; do
  tag=$(basename $v .so)
  raw=$(mktemp -d /tmp/luc_XXXX)
  if [ $v = default ]; then unset IADMM_LIB_PATH; else export IADMM_LIB_PATH=$PWD/$v; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$raw" -o run -- python3 tools/profile_lu.py \
    > gpurun_out/r03c/$tag.log 2>&1 || { echo "rocprof $tag failed"; exit 1; }
  cp "$(find "$raw" -name "*kernel_stats.csv" | head -1)" gpurun_out/r03c/${tag}_kernel_stats.csv
  rm -rf "$raw"
done
unset IADMM_LIB_PATH
for f in gpurun_out/r03c/*_kernel_stats.csv; do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "lu_" in r["Name"] or "kkt_assemble" in r["Name"]:
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} total {float(r["TotalDurationNs"])/1e6:8.2f} ms avg {float(r["AverageNs"])/1e3:9.1f} us')
PY
done
