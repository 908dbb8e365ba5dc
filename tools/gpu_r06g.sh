#!/bin/bash
# r06: capture probe variants 9/10 (origin-only forks: the batch split, the reworked look-ahead) on torch's
# HIP runtime, then the LU graph-capture tests with the captured look-ahead / split; sched_bwd batch loads
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -shared -fPIC -DPROBE_LIB tools/capture_probe.hip -o /tmp/probe.so || exit 5
for v in 1 9 10; do
  timeout -k 10 120 python3 -u tools/capture_probe_torch.py /tmp/probe.so $v >> gpurun_out/r06g_capture_probe_torchrt.log 2>&1
  rc=$?
  echo "variant $v rc=$rc" >> gpurun_out/r06g_capture_probe_torchrt.log
  [ $rc -ne 0 ] && { grep -v amdgpu.ids gpurun_out/r06g_capture_probe_torchrt.log | tail -20; exit 6; }
done
grep -v amdgpu.ids gpurun_out/r06g_capture_probe_torchrt.log | grep "variant"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_abi_concurrency_gpu.py tests/test_train_gpu.py tests/test_window_grads_gpu.py > gpurun_out/r06g_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r06g_tests.log | tail -30
exit $rc
