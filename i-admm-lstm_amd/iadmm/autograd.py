"""torch.autograd bindings of the HIP kernels: training through the unrolled solve.

``IterationFn`` is one I-ADMM-LSTM iteration (models/lstm.py:47-96) as an autograd Function whose
forward runs the same three kernels as inference and whose backward runs the hand-written
backward kernels (csrc/train.hip, csrc/gemm.hip); ``LossFn`` is the unsupervised loss of
utils.py:68-71.  Chained by torch's autograd engine over the T iterations of a truncation window
(main.py:336-350), they give the reference's TBPTT gradients for all 16 parameters.

Saved per iteration: the iteration's inputs (x, y, z, xv, H, C), g = K^T(K xv - b~), the residual
r = K xv - b~ and xv'.  The gate pre-activations are recomputed on MFMA in the backward instead
of being stored (4 [B*N, h] tensors per iteration).
"""
from __future__ import annotations

import torch

from . import ops
from .solver import PARAM_NAMES

GATES = "ifou"


class IterationFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, x, y, z, xv, H, C, *params):
        t, num_ineq, sigma, data, packed = meta
        p = dict(zip(PARAM_NAMES, params))
        Q, pv, A0, zl, zu = data
        B, n = x.shape
        m = y.shape[1]
        h = H.shape[-1]
        det = lambda a: a.detach().contiguous()  # noqa: E731
        scal = ops.schedule(det(p["rho"]), det(p["alpha"]), t)
        r = ops.empty(B, n + m, like=x)
        btild = ops.empty(B, n + m, like=x)
        rho_vec = ops.empty(B, m, like=x)
        g = ops.kkt_resgrad(Q, A0, pv, x, y, z, xv, sigma, scal, num_ineq, btild=btild, rho_vec=rho_vec, r_out=r)
        Upk, Wx = packed.get({k: v.detach() for k, v in p.items()}, h)
        Hn, Cn, part = ops.lstm_cell(H, C, xv, g, Upk, Wx)
        xvo, xo, yo, zo = ops.admm_update(n, m, num_ineq, part, det(p["b_h"]), xv, x, y, z, zl, zu, scal)
        ctx.save_for_backward(x, y, z, xv, H, C, g, r, xvo, scal, *params)
        ctx.meta = meta
        ctx.extra = (btild, rho_vec)
        ctx.mark_non_differentiable(btild, rho_vec)
        return xo, yo, zo, xvo, Hn, Cn, btild, rho_vec

    @staticmethod
    def backward(ctx, dxo, dyo, dzo, dxvo, dHn, dCn, _db, _dr):
        x, y, z, xv, H, C, g, r, xvo, scal, *params = ctx.saved_tensors
        t, num_ineq, sigma, data, packed = ctx.meta
        p = dict(zip(PARAM_NAMES, params))
        Q, pv, A0, zl, zu = data
        B, n = x.shape
        m = y.shape[1]
        h = H.shape[-1]
        M = B * (n + m)
        c = lambda a: None if a is None else a.contiguous()  # noqa: E731
        # 1. update: x', z', y', xv' -> dq and partial input adjoints
        dx, dy, dz, dxv, dq, upd_part = ops.admm_update_bwd(n, m, num_ineq, x, y, z, xvo, zl, zu, scal, c(dxo),
                                                             c(dyo), c(dzo), c(dxvo))
        # 2. cell: recompute gates, dP, dC, d(in) partials, W_h slabs
        Upk, Wx = packed.get({k: v.detach() for k, v in p.items()}, h)
        dC, dP, whslab, inpart = ops.lstm_cell_bwd(H, C, xv, g, Upk, Wx, dq, c(dHn), c(dCn))
        # 3. dH = dP U_cat^T ; [dU ; dW ; db] = [H, xv, g, 1]^T dP
        Ucat_pk = packed.get_ucat_packed({k: v.detach() for k, v in p.items()}, h)     # [h, 4h], tiled
        dH = ops.gemm_nt_packed(dP, Ucat_pk, h).reshape(H.shape)
        dUcat = ops.gemm_tn(H.reshape(M, h), dP)
        X3 = torch.stack([xv.reshape(M), g.reshape(M), torch.ones(M, device=x.device)], dim=1).contiguous()
        dW3 = ops.gemm_tn(X3, dP, rows_per_split=512)                                 # [3, 4h], streaming
        dWh = ops.slab_reduce(whslab).reshape(h, 1)
        # 4. d(in) -> d(xv), dg ; 5. KKT backward
        dg = ops.in_reduce(inpart, dxv)
        kkt_ds = ops.kkt_bwd(Q, A0, xv, y, r, dg.reshape(B, n + m), sigma, scal, num_ineq, dxv, dx, dy, dz)
        # 6. schedule scalars and b_h
        drho = torch.zeros_like(p["rho"])
        dalpha = torch.zeros_like(p["alpha"])
        dbh = torch.zeros_like(p["b_h"])
        ops.sched_bwd(p["rho"].detach().contiguous(), p["alpha"].detach().contiguous(), t, upd_part, kkt_ds,
                      drho, dalpha, dbh)
        grads = {}
        for gi, k in enumerate(GATES):
            sl = slice(gi * h, (gi + 1) * h)
            grads["W_" + k] = dW3[0:2, sl].contiguous()
            grads["U_" + k] = dUcat[:, sl].contiguous()
            grads["b_" + k] = dW3[2, sl].contiguous()
        grads.update(W_h=dWh, b_h=dbh, rho=drho, alpha=dalpha)
        pgrads = [grads[k] if ctx.needs_input_grad[7 + i] else None for i, k in enumerate(PARAM_NAMES)]
        return (None, dx, dy, dz, dxv, dH, dC, *pgrads)


class LossFn(torch.autograd.Function):
    """(||A0 x - z||, ||Q x + p + A0^T y||) per instance (utils.py:68-71); the data (Q, p, A0) is
    constant (no gradient)."""

    @staticmethod
    def forward(ctx, x, y, z, data):
        Q, pv, A0 = data
        # one sweep (row-block split: fills the chip at the micro-batch); the gradient sweep runs in
        # backward
        pr, du, _, _, _ = ops.loss_grad(Q, pv, A0, x, y, z, want_grad=False)
        ctx.save_for_backward(x, y, z)
        ctx.data = data
        return pr, du

    @staticmethod
    def backward(ctx, dpr, ddu):
        x, y, z = ctx.saved_tensors
        Q, pv, A0 = ctx.data
        cp = dpr.contiguous() if dpr is not None else torch.zeros(x.shape[0], device=x.device)
        cd = ddu.contiguous() if ddu is not None else torch.zeros(x.shape[0], device=x.device)
        _, _, dx, dy, dz = ops.loss_grad(Q, pv, A0, x, y, z, cp, cd)
        return dx, dy, dz, None
