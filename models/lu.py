"""Drop-in ``models.lu.LU`` (reference: models/lu.py:4-47): Stage II exact ADMM iteration.

The batched LU factor/solve kernels (iadmm_lu_factor / iadmm_lu_solve) are the next milestone;
until they land this module refuses to run rather than falling back to a library or the CPU.
"""
import torch.nn as nn

import iadmm_path  # noqa: F401


class LU(nn.Module):
    ALPHA = 1.6  # models/lu.py:24

    def __init__(self, device):
        super().__init__()
        self.device = device

    def name(self):
        return 'torch_solver'

    def forward(self, rho_vec, x, y, z, xv, sigma, A_tild, lu, piv, **kwargs):
        raise NotImplementedError("Stage II batched LU kernels are not built yet")
