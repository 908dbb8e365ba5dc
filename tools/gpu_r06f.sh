#!/bin/bash
# r06: panels' staged loads double-buffered for real (inline-asm stage reads) -- LU tests, A/B against
# the previous build; recipe epoch time with cached synthetic instances; then the capture probe's
# stream patterns on torch's bundled HIP runtime (probe library loaded after torch; last: may crash)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_stage2_gpu.py tests/test_abi_concurrency_gpu.py tests/test_lu_hbm_gpu.py > gpurun_out/r06f_lu_tests.log 2>&1 || { tail -n 40 gpurun_out/r06f_lu_tests.log; exit 1; }
tail -n 2 gpurun_out/r06f_lu_tests.log
timeout -k 10 600 python3 tools/lu_ab.py --libs tools/var_lu_before.so i-admm-lstm_amd/iadmm/libiadmm.so \
  tools/var_lu_before.so i-admm-lstm_amd/iadmm/libiadmm.so --batch 1024 --N 2000 > gpurun_out/r06f_lu_ab_panel.txt 2>&1 || exit 2
grep '^{' gpurun_out/r06f_lu_ab_panel.txt | cut -c1-200
bash tools/train_reference_recipe.sh r06u 3 || exit 3
grep -h "Epoch" gpurun_out/r06u_recipe/train.log | head -12
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -shared -fPIC -DPROBE_LIB tools/capture_probe.hip -o /tmp/probe.so || exit 5
for v in 1 2 3 4 5 6 7 8; do
  timeout -k 10 120 python3 -u tools/capture_probe_torch.py /tmp/probe.so $v >> gpurun_out/r06f_capture_probe_torchrt.log 2>&1
  rc=$?
  echo "variant $v rc=$rc" >> gpurun_out/r06f_capture_probe_torchrt.log
  [ $rc -ne 0 ] && break
done
grep -v amdgpu.ids gpurun_out/r06f_capture_probe_torchrt.log | tail -30
exit 0
