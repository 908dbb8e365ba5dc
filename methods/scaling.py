"""Drop-in ``methods.scaling.Scaling`` (reference: methods/scaling.py:5-119), HIP-backed.

``scale_data`` runs all Ruiz rounds in one gfx950 launch (iadmm_ruiz_scale, O(n^2) per
instance instead of the reference's dense-diagonal bmm, O(n^3)), keeping the reference's
rounding order so the scaled data match element for element.  The scaling factors are kept as
vectors (``d``, ``e``, ``c_vec``); the reference's dense attributes ``D``, ``D_inv``, ``E``,
``Einv`` ([B,k,k]) and ``c``, ``cinv`` ([B,1,1]) are materialised on first access for callers
that ``torch.bmm`` with them (main.py:876-878).
"""
import torch

import iadmm_path  # noqa: F401
from iadmm import ops


class Scaling(object):
    MIN_SCALING = 1e-04  # methods/scaling.py:12-13 (fixed in the kernel)
    MAX_SCALING = 1e04

    def __init__(self, num_var, num_constr, scaling_ites, device):
        self.n = num_var
        self.m = num_constr
        self.device = device
        self.scaling_ites = scaling_ites
        self.d = self.e = self.c_vec = None

    def scale_data(self, Q, p, A0, lb, ub):
        f = lambda a: a.detach().float().contiguous()  # noqa: E731
        Qs, ps, As, lbs, ubs, d, e, c = ops.ruiz_scale(f(Q), f(p), f(A0), f(lb), f(ub), self.scaling_ites)
        self.d, self.e, self.c_vec = d, e, c
        return Qs, ps, As, lbs, ubs

    # --- reference attribute surface (dense, materialised lazily)
    @property
    def D(self):
        return torch.diag_embed(self.d)

    @property
    def D_inv(self):
        return torch.diag_embed(torch.reciprocal(self.d))

    @property
    def E(self):
        return torch.diag_embed(self.e)

    @property
    def Einv(self):
        return torch.diag_embed(torch.reciprocal(self.e))

    @property
    def c(self):
        return self.c_vec.reshape(-1, 1, 1)

    @property
    def cinv(self):
        return 1.0 / self.c

    def unscale(self, x, y, z):
        """x = D x, y = (c^-1 E) y, z = E^-1 z without dense matrices (main.py:1025-1027)."""
        B = x.shape[0]
        xo, yo, zo = ops.unscale(self.d, self.e, self.c_vec, x.reshape(B, -1).contiguous(),
                                 y.reshape(B, -1).contiguous(), z.reshape(B, -1).contiguous())
        return xo.unsqueeze(-1), yo.unsqueeze(-1), zo.unsqueeze(-1)
