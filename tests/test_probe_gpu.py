"""Box-ceiling probes (csrc/probe.hip, bench.py box_ceiling): the register-only fp32 MFMA stream and
the float4 HBM copy run through the C-ABI and report rates in the physically possible range of an
MI355X (below the spec peaks, above half of them), and the copy moves the bytes."""
import pytest
import torch

import iadmm_path  # noqa: F401

pytestmark = pytest.mark.gpu


def test_box_ceiling_rates_are_plausible():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import bench
    box = bench.box_ceiling(torch.cuda.current_device())
    print("[box ceiling]", {k: v for k, v in box.items() if k != "method"})
    assert box["copy_checked"]
    assert 0.5 * bench.FP32_MFMA_PEAK_TFLOPS < box["mfma_f32_tflops"] < 1.02 * bench.FP32_MFMA_PEAK_TFLOPS
    assert 0.4 * bench.HBM_PEAK_GBS < box["hbm_copy_gbs"] < 1.0 * bench.HBM_PEAK_GBS
    assert 0.4 * bench.HBM_PEAK_GBS < box["hbm_read_gbs"] < 1.0 * bench.HBM_PEAK_GBS
    assert box["hbm_gbs"] == max(box["hbm_copy_gbs"], box["hbm_read_gbs"])


def test_probe_arguments_rejected():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from iadmm import _abi
    L = _abi.lib()
    x = torch.empty(64, device="cuda")
    assert L.iadmm_probe_mfma(0, 10, x.data_ptr(), None) == -1
    assert L.iadmm_probe_copy(12, x.data_ptr(), x.data_ptr(), None) == -3
    assert L.iadmm_probe_copy(16, None, x.data_ptr(), None) == -1
    assert L.iadmm_probe_read(16, x.data_ptr(), x.data_ptr(), 0, 8, None) == -1
    assert L.iadmm_probe_read(16, x.data_ptr(), x.data_ptr(), 4, 4, None) == -1
    assert L.iadmm_probe_read(12, x.data_ptr(), x.data_ptr(), 4, 8, None) == -3
