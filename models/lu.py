"""Drop-in ``models.lu.LU`` (reference: models/lu.py:4-47): Stage II exact ADMM iteration.

First call (``lu is None and piv is None``): the dense K is assembled on the device
(iadmm_kkt_assemble) with the caller's per-row ``rho_vec``, factored in place by the batched
blocked LU kernel (iadmm_lu_factor) and solved (iadmm_lu_solve); later calls reuse (lu, piv).
The x/z/y update runs with the fixed alpha = 1.6 relaxation on x AND z (iadmm_admm_update,
relax_z).  Returns the reference's 8-tuple; ``A_tild`` is a lazy KKT operator carrying the same
rho (``torch.bmm(A_tild, xv)`` works, ``.dense()`` materialises it) and ``piv`` holds 1-based
int32 row interchanges like ``torch.lu`` / LAPACK, so (lu, piv) also feed ``torch.linalg.lu_solve``.
A singular K raises like ``torch.lu`` does.
"""
import torch
import torch.nn as nn

import iadmm_path  # noqa: F401
from iadmm import ops
from iadmm.kktop import KKTOperator
from iadmm.solver import fixed_alpha_scal


class LU(nn.Module):
    ALPHA = 1.6  # models/lu.py:24

    def __init__(self, device):
        super().__init__()
        self.device = device
        self._scal = None

    def name(self):
        return 'torch_solver'

    def forward(self, rho_vec, x, y, z, xv, sigma, A_tild, lu, piv, **kwargs):
        Q, p, A0, zl, zu = (kwargs[k] for k in ("Q", "p", "A0", "zl", "zu"))
        f = lambda a: a.detach().float().contiguous()  # noqa: E731
        B, n = x.shape[0], x.shape[1]
        m = y.shape[1]
        Q, A0 = f(Q), f(A0)
        rho = f(rho_vec).reshape(B, m)
        xf, yf, zf = f(x).reshape(B, n), f(y).reshape(B, m), f(z).reshape(B, m)
        b = ops.kkt_rhs(f(p).reshape(B, n), xf, yf, zf, float(sigma), rho_rows=rho)
        if lu is None and piv is None:
            K = ops.kkt_assemble(Q, A0, float(sigma), None, 0, rho_rows=rho)
            lu, piv, info = ops.lu_factor(K)
            bad = int(info.max())  # one host read per factorisation, as torch.lu's error check
            if bad:
                raise RuntimeError(f"LU factorisation: U({bad},{bad}) is exactly zero (singular KKT matrix)")
            A_tild = KKTOperator(Q, A0, float(sigma), None, 0, rho_rows=rho)
        xs = ops.lu_solve(lu, piv, b)
        if self._scal is None or self._scal.device != xs.device:
            self._scal = fixed_alpha_scal(self.ALPHA, xs.device)
        xvo, xo, yo, zo = ops.admm_update(n, m, 0, None, None, xs, xf, yf, zf, f(zl).reshape(B, m),
                                          f(zu).reshape(B, m), self._scal, relax_z=True, rho_rows=rho)
        return (xo.unsqueeze(-1), yo.unsqueeze(-1), zo.unsqueeze(-1), xvo.unsqueeze(-1), A_tild,
                b.unsqueeze(-1), lu, piv)
