#!/bin/bash
# r04 session 4: new / changed GPU tests (probes, Stage-II envelopes, LU, training), then a default bench
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh r04g 1000 tests/test_probe_gpu.py tests/test_stage2_gpu.py "tests/test_k100_gpu.py::test_stage2_after_k100_vs_oracle" "tests/test_config4_gpu.py::test_config4_stage2_vs_oracle" tests/test_train_gpu.py tests/test_train_split_gpu.py || exit $?
grep -E "^\[stage2|PASS|FAIL|passed|failed|box ceiling" gpurun_out/r04g_tests.log | tail -60
