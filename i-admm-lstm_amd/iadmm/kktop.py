"""Lazy KKT operator: what the drop-in ``LSTM.forward`` returns as ``A_tild``.

The reference returns the dense K [B,N,N] (models/lstm.py:96; 16.4 GB at the bench config) and
``main.py`` only uses it as ``torch.bmm(A_tild, xv)`` for ``ls_res`` (main.py:952).  This object
keeps (Q, A0, sigma, rho) and implements ``torch.bmm(op, v)``, ``op.permute(0, 2, 1)``,
``op @ v`` and ``op.bmm(v)`` with the implicit-K HIP kernel; ``dense()`` materialises K.
"""
from __future__ import annotations

import torch

from . import ops


class KKTOperator:
    def __init__(self, Q, A0, sigma, scal, num_ineq, transposed=False, rho_rows=None):
        self.Q, self.A0, self.sigma, self.scal = Q, A0, float(sigma), scal
        self.num_ineq = int(num_ineq)
        self.transposed = transposed
        self.rho_rows = rho_rows  # explicit per-row rho (Stage II); else two-class rho from scal
        B, n = Q.shape[0], Q.shape[1]
        N = n + A0.shape[1]
        self.shape = torch.Size((B, N, N))
        self.device = Q.device
        self.dtype = Q.dtype

    # -- tensor-like surface used by reference-style callers
    def permute(self, *dims):
        dims = tuple(dims[0]) if len(dims) == 1 and isinstance(dims[0], (tuple, list)) else dims
        if tuple(dims) != (0, 2, 1):
            raise NotImplementedError("KKTOperator only supports permute(0, 2, 1)")
        return KKTOperator(self.Q, self.A0, self.sigma, self.scal, self.num_ineq, not self.transposed,
                           self.rho_rows)

    def transpose(self, d0, d1):
        if {d0 % 3, d1 % 3} != {1, 2}:
            raise NotImplementedError("KKTOperator only transposes its matrix dims")
        return self.permute(0, 2, 1)

    @property
    def mT(self):
        return self.permute(0, 2, 1)

    def size(self, dim=None):
        return self.shape if dim is None else self.shape[dim]

    def dim(self):
        return 3

    def bmm(self, v):
        if v.dim() != 3 or v.shape[-1] != 1:
            raise NotImplementedError("KKTOperator.bmm supports [B,N,1] right-hand sides")
        out = ops.kkt_matvec(self.Q, self.A0, v.reshape(v.shape[0], -1).contiguous(), self.sigma,
                             self.scal, self.num_ineq, transpose=self.transposed, rho_rows=self.rho_rows)
        return out.unsqueeze(-1)

    __matmul__ = bmm

    def dense(self):
        K = ops.kkt_assemble(self.Q, self.A0, self.sigma, self.scal, self.num_ineq, rho_rows=self.rho_rows)
        return K.transpose(1, 2).contiguous() if self.transposed else K

    def to_dense(self):
        return self.dense()

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in (torch.bmm, torch.matmul, torch.Tensor.bmm, torch.Tensor.matmul) and isinstance(args[0], cls):
            return args[0].bmm(args[1])
        if func in (torch.Tensor.permute, torch.permute) and isinstance(args[0], cls):
            return args[0].permute(*args[1:])
        raise NotImplementedError(f"KKTOperator does not implement {getattr(func, '__name__', func)}; "
                                  "call .dense() for an explicit K")
