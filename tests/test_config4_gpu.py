"""BASELINE config-4 instance shape (n=5000, m=2500+2500, h=2048) on the GPU: exercises the
large-instance kernel paths (24 column groups per lane, > 64 KiB dynamic LDS for the KKT / Ruiz /
metric kernels, h = 2048 cell tiles) against the CPU oracle on one instance, T = 2.
Same tolerances as the bench-shape test (tests/test_fullsize_gpu.py)."""
import numpy as np
import pytest
import torch

import iadmm_path  # noqa: F401
from oracle import iadmm_oracle as orc

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-30))


@pytest.mark.timeout(900)  # the CPU oracle at n + m = 10000, h = 2048 alone takes minutes on a busy host
def test_config4_shape_vs_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from iadmm import data, solver
    n, mi, me, h, T = 5000, 2500, 2500, 2048, 2
    d = data.make_qp_batch(n, mi, me, 1, first_index=0, device="cuda")
    params = data.init_lstm_params(h, 200, device="cuda")
    cpu = {k: v.cpu() for k, v in d.items()}  # before the in-place scaling below
    with torch.no_grad():
        out = solver.solve(params, d["Q"], d["p"], d["A0"], d["zl"], d["zu"], mi, me, T, 6e-6, keep_unscaled=False)
    torch.cuda.synchronize()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    with torch.no_grad():
        ref = orc.solve({k: v.cpu() for k, v in params.items()}, cpu["Q"], cpu["p"], cpu["A0"], cpu["zl"],
                        cpu["zu"], mi, me, T, 6e-6, h)
    assert rel_l2(out["D"], torch.diagonal(ref["scaling"]["D"], dim1=1, dim2=2)) < 1e-6
    for k in ("x", "z", "xv"):
        assert rel_l2(out[k], ref[k]) < 1e-4, k
    assert rel_l2(out["y"], ref["y"]) < 5e-3
    assert rel_l2(out["H"], ref["H"]) < 1e-4
    assert rel_l2(out["C"], ref["C"]) < 1e-4
    np.testing.assert_allclose(out["primal"].cpu().numpy(), ref["primal"].numpy(), rtol=1e-4)
    np.testing.assert_allclose(out["dual"].cpu().numpy(), ref["dual"].numpy(), rtol=1e-4)
