#!/bin/bash
# r06: LU batch-split stagger A/B; the recipe's epoch time at HEAD (main.py train mode, batch 2, fresh run for two minutes), then the
# capture probe's stream patterns under the HIP runtime that python processes load (torch's bundled
# libamdhip64, ROCm 7.0.2) instead of the system 7.2 one (last: may crash)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/lu_ab.py --libs i-admm-lstm_amd/iadmm/libiadmm.so tools/var_stagger1.so tools/var_stagger2.so \
  i-admm-lstm_amd/iadmm/libiadmm.so tools/var_stagger1.so tools/var_stagger2.so --batch 1024 --N 2000 > gpurun_out/r06e_lu_ab_stagger.txt 2>&1 || exit 1
grep lib gpurun_out/r06e_lu_ab_stagger.txt | cut -c1-300
bash tools/train_reference_recipe.sh r06t 2 || exit 1
grep -h "Epoch" gpurun_out/r06t_recipe/train.log | head -12
TL=$(python3 -c "import torch, os; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/capture_probe.hip -o /tmp/capture_probe || exit 5
for v in 1 2 3 4 5 6 7 8; do
  LD_LIBRARY_PATH=$TL timeout -k 10 60 /tmp/capture_probe $v >> gpurun_out/r06e_capture_probe_torchrt.log 2>&1
  rc=$?
  echo "variant $v rc=$rc" >> gpurun_out/r06e_capture_probe_torchrt.log
  [ $rc -ne 0 ] && break
done
LD_LIBRARY_PATH=$TL ldd /tmp/capture_probe | grep amdhip >> gpurun_out/r06e_capture_probe_torchrt.log
tail -n 30 gpurun_out/r06e_capture_probe_torchrt.log
exit 0
