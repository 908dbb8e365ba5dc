#!/bin/bash
# r04 session 8: the K = 100 parity test (trained weights) for candidate checkpoints of the recipe run
# (epoch-39's save measured a primal-history error of 6.5e-4 against the 1e-4 bound)
set -o pipefail
mkdir -p gpurun_out
cp checkpoints/QP_1000_500_500_100_800.pth /tmp/ckpt_head.pth
for e in e55; do
  cp variants/ckpt/$e.pth checkpoints/QP_1000_500_500_100_800.pth
  timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s "tests/test_k100_gpu.py::test_k100_vs_oracle[trained]" > gpurun_out/r04ck55_$e.log 2>&1
  rc=$?
  echo "$e rc=$rc"; grep "\[k100" gpurun_out/r04ck55_$e.log | cut -c1-200
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
cp /tmp/ckpt_head.pth checkpoints/QP_1000_500_500_100_800.pth
