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

# Optional solver.Timer: hipEvent spans ("k:cell_fwd", "k:cell_bwd", "k:dH", "k:dU") around the
# training kernels on the current stream (bench.py's training record; None = no events).
TIMER = None


def _span(name):
    return TIMER.start(name) if TIMER is not None else None


def _end(tok):
    if tok is not None:
        TIMER.stop(tok)


class WindowGrads:
    """Parameter-gradient accumulators shared by the IterationFn nodes of one chain of iterations (a
    TBPTT window: each iteration's H comes out of the previous one's node).

    r06: every node used to return its 16 parameter gradients to autograd, whose input buffers then
    summed the T contributions per parameter (a 10-MB add per U gate, an add and a gather copy per
    tensor per iteration: ~20 launches per iteration, 8 % of a batch-2 window).  Now each node adds
    its contributions straight into these buffers -- through the reductions that produce them
    (slab reduce with accumulate, the schedule backward's +=) -- and returns None for the
    parameters; the chain's first node (``owner``), whose backward runs after every later node's,
    returns the sums.  Autograd's input buffer kept the first contribution as is and added the next
    ones in execution order (t = T-1 down to 0); the buffers here start from the first reduction
    (accumulate = 0) and add in the same order, so the gradients are the same sums in the same order
    (the per-iteration slices of dU_cat / dW3 are taken once, at the end)."""

    __slots__ = ("key", "dUcat", "dW3", "dWh", "drho", "dalpha", "dbh")

    def __init__(self, key):
        self.key = key
        self.reset()

    def reset(self):
        self.dUcat = self.dW3 = self.dWh = self.drho = self.dalpha = self.dbh = None


def window_grads_for(H, params):
    """(WindowGrads, owner) for an iteration whose hidden state is H: the chain's accumulators when H
    came out of an IterationFn of the same parameters, else new ones owned by this iteration."""
    key = tuple(id(q) for q in params)
    prev = getattr(H.grad_fn, "iadmm_acc", None) if H.grad_fn is not None else None
    if prev is not None and prev.key == key:
        return prev, False
    return WindowGrads(key), True


class IterationFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, meta, x, y, z, xv, H, C, *params):
        t, num_ineq, sigma, data, packed, acc, owner = meta
        ctx.iadmm_acc, ctx.iadmm_owner = acc, owner
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
        k = _span("k:cell_fwd")
        Hn, Cn, part = ops.lstm_cell(H, C, xv, g, Upk, Wx)
        _end(k)
        xvo, xo, yo, zo = ops.admm_update(n, m, num_ineq, part, det(p["b_h"]), xv, x, y, z, zl, zu, scal)
        ctx.save_for_backward(x, y, z, xv, H, C, g, r, xvo, scal, *params)
        ctx.meta = meta
        ctx.extra = (btild, rho_vec)
        ctx.mark_non_differentiable(btild, rho_vec)
        return xo, yo, zo, xvo, Hn, Cn, btild, rho_vec

    @staticmethod
    def backward(ctx, dxo, dyo, dzo, dxvo, dHn, dCn, _db, _dr):
        x, y, z, xv, H, C, g, r, xvo, scal, *params = ctx.saved_tensors
        t, num_ineq, sigma, data, packed, _, _ = ctx.meta
        acc = ctx.iadmm_acc
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
        k = _span("k:cell_bwd")
        dC, dP, whslab, inpart = ops.lstm_cell_bwd(H, C, xv, g, Upk, Wx, dq, c(dHn), c(dCn))
        _end(k)
        # 3. dH = dP U_cat^T ; [dU ; dW ; db] = [H, xv, g, 1]^T dP
        Ucat_pk = packed.get_ucat_packed({k: v.detach() for k, v in p.items()}, h)     # [h, 4h], tiled
        k = _span("k:dH")
        dH = ops.gemm_nt_packed(dP, Ucat_pk, h).reshape(H.shape)
        _end(k)
        need = {k: ctx.needs_input_grad[7 + i] for i, k in enumerate(PARAM_NAMES)}
        k = _span("k:dU")
        if any(need["U_" + q] for q in GATES):
            if acc.dUcat is None:
                acc.dUcat = ops.gemm_tn(H.reshape(M, h), dP)
            else:
                ops.gemm_tn(H.reshape(M, h), dP, out=acc.dUcat, accumulate=True)
        _end(k)
        if any(need[q + g_] for q in ("W_", "b_") for g_ in GATES):
            X3 = torch.stack([xv.reshape(M), g.reshape(M), torch.ones(M, device=x.device)], dim=1).contiguous()
            if acc.dW3 is None:
                acc.dW3 = ops.gemm_tn(X3, dP)                                          # [3, 4h], streaming
            else:
                ops.gemm_tn(X3, dP, out=acc.dW3, accumulate=True)
        if need["W_h"]:
            if acc.dWh is None:
                acc.dWh = ops.slab_reduce(whslab)
            else:
                ops.slab_reduce(whslab, out=acc.dWh, accumulate=True)
        # 4. d(in) -> d(xv), dg ; 5. KKT backward
        dg = ops.in_reduce(inpart, dxv)
        kkt_ds = ops.kkt_bwd(Q, A0, xv, y, r, dg.reshape(B, n + m), sigma, scal, num_ineq, dxv, dx, dy, dz)
        # 6. schedule scalars and b_h (iadmm_sched_bwd adds into its outputs)
        if acc.drho is None:
            acc.drho = torch.zeros_like(p["rho"])
            acc.dalpha = torch.zeros_like(p["alpha"])
            acc.dbh = torch.zeros_like(p["b_h"])
        ops.sched_bwd(p["rho"].detach().contiguous(), p["alpha"].detach().contiguous(), t, upd_part, kkt_ds,
                      acc.drho, acc.dalpha, acc.dbh)
        pgrads = [None] * len(PARAM_NAMES)
        if ctx.iadmm_owner:  # the chain's first iteration: every later node has added its share
            grads = dict(W_h=None if acc.dWh is None else acc.dWh.reshape(h, 1), b_h=acc.dbh, rho=acc.drho,
                         alpha=acc.dalpha)
            for gi, q in enumerate(GATES):
                sl = slice(gi * h, (gi + 1) * h)
                grads["W_" + q] = None if acc.dW3 is None else acc.dW3[0:2, sl].contiguous()
                grads["U_" + q] = None if acc.dUcat is None else acc.dUcat[:, sl].contiguous()
                grads["b_" + q] = None if acc.dW3 is None else acc.dW3[2, sl].contiguous()
            pgrads = [grads[k] if ctx.needs_input_grad[7 + i] else None for i, k in enumerate(PARAM_NAMES)]
            acc.reset()  # (the buffers now belong to autograd; a retained graph's next backward starts anew)
        return (None, dx, dy, dz, dxv, dH, dC, *pgrads)


class LossFn(torch.autograd.Function):
    """(||A0 x - z||, ||Q x + p + A0^T y||) per instance (utils.py:68-71).  x, y, z: the training
    loss's inputs (iadmm_loss_grad_split sweeps); Q, p, A0: data, differentiable too when they
    require grad (rank-1 iadmm_bger terms from the two residual vectors)."""

    @staticmethod
    def forward(ctx, x, y, z, Q, pv, A0):
        # one sweep (row-block split: fills the chip at the micro-batch); the gradient sweep runs in
        # backward
        pr, du, _, _, _ = ops.loss_grad(Q, pv, A0, x, y, z, want_grad=False)
        ctx.save_for_backward(x, y, z, Q, pv, A0, pr, du)
        return pr, du

    @staticmethod
    def backward(ctx, dpr, ddu):
        x, y, z, Q, pv, A0, pr, du = ctx.saved_tensors
        cp = dpr.contiguous() if dpr is not None else torch.zeros(x.shape[0], device=x.device)
        cd = ddu.contiguous() if ddu is not None else torch.zeros(x.shape[0], device=x.device)
        dx = dy = dz = dQ = dp = dA = None
        if any(ctx.needs_input_grad[:3]):
            _, _, dx, dy, dz = ops.loss_grad(Q, pv, A0, x, y, z, cp, cd)
        if any(ctx.needs_input_grad[3:]):
            # unit residual directions scaled by the upstream coefficients (norm' = r / ||r||; a
            # zero residual gives 0 like torch's vector_norm backward)
            r = ops.bmv(A0, x) - z
            d = ops.bmv(Q, x) + pv + ops.bmv_t(A0, y)
            wr = (r * (cp / pr).nan_to_num(0.0, 0.0, 0.0).reshape(-1, 1)).contiguous()
            wd = (d * (cd / du).nan_to_num(0.0, 0.0, 0.0).reshape(-1, 1)).contiguous()
            if ctx.needs_input_grad[3]:
                dQ = ops.bger(wd, x)
            if ctx.needs_input_grad[4]:
                dp = wd
            if ctx.needs_input_grad[5]:
                dA = ops.bger(wr, x)
                ops.bger(y, wd, out=dA, accumulate=True)
        return dx, dy, dz, dQ, dp, dA


# ----------------------------------------------------------------------------- reporting metrics
# utils.py:53-60 are plain torch expressions in the reference, so autograd reaches x and the data.
# Their backward here: the matvecs on iadmm_bmv / iadmm_bmv_t, the matrix gradients (rank 1 per
# instance) on iadmm_bger; the [B, rows] vector algebra in between is elementwise.  The gradient
# conventions are torch's: clamp(min=0) passes where its input >= 0, abs' derivative is sgn (0 at 0).

def _vec(a):
    return a.reshape(a.shape[0], -1).contiguous()


class ObjFn(torch.autograd.Function):
    """0.5 x^T Q x + p^T x per instance (utils.py:53-54): x [B,n], Q [B,n,n], p [B,n] -> [B]."""

    @staticmethod
    def forward(ctx, x, Q, p):
        B, n = x.shape
        zeros = x.new_zeros(B, 0)
        obj, _, _ = ops.metrics(Q, p, Q.new_zeros(B, 0, n), x, zeros, zeros)
        ctx.save_for_backward(x, Q, p)
        return obj

    @staticmethod
    def backward(ctx, g):
        x, Q, p = ctx.saved_tensors
        g = g.reshape(-1, 1).contiguous()
        hx = (0.5 * g) * x                   # d/d(Qx) of 0.5 x^T (Qx)
        dx = dQ = dp = None
        if ctx.needs_input_grad[0]:
            dx = ops.bmv(Q, x) * (0.5 * g) + ops.bmv_t(Q, hx.contiguous()) + g * p
        if ctx.needs_input_grad[1]:
            dQ = ops.bger(hx.contiguous(), x)
        if ctx.needs_input_grad[2]:
            dp = g * x
        return dx, dQ, dp


class IneqDistFn(torch.autograd.Function):
    """clamp(G x - c, 0) (utils.py:56-57): x [B,n], G [B,mi,n], c [B,mi] -> [B,mi]."""

    @staticmethod
    def forward(ctx, x, G, c):
        pre = ops.bmv(G, x) - c
        ctx.save_for_backward(x, G, pre >= 0)
        return torch.clamp(pre, min=0)

    @staticmethod
    def backward(ctx, w):
        x, G, mask = ctx.saved_tensors
        w = (w * mask).contiguous()
        dx = ops.bmv_t(G, w) if ctx.needs_input_grad[0] else None
        dG = ops.bger(w, x) if ctx.needs_input_grad[1] else None
        dc = -w if ctx.needs_input_grad[2] else None
        return dx, dG, dc


class EqDistFn(torch.autograd.Function):
    """|b - A x| (utils.py:59-60): x [B,n], A [B,me,n], b [B,me] -> [B,me]."""

    @staticmethod
    def forward(ctx, x, A, b):
        r = b - ops.bmv(A, x)
        ctx.save_for_backward(x, A, torch.sgn(r))
        return r.abs()

    @staticmethod
    def backward(ctx, w):
        x, A, s = ctx.saved_tensors
        ws = (w * s).contiguous()               # d/dr
        dx = -ops.bmv_t(A, ws) if ctx.needs_input_grad[0] else None
        dA = -ops.bger(ws, x) if ctx.needs_input_grad[1] else None
        db = ws if ctx.needs_input_grad[2] else None
        return dx, dA, db


class BmvFn(torch.autograd.Function):
    """Differentiable batched matvec M x (M [B,R,C], x [B,C] -> [B,R]): iadmm_bmv forward,
    iadmm_bmv_t / iadmm_bger backward.  The building block of utils.aug_lagr under grad."""

    @staticmethod
    def forward(ctx, M, x):
        ctx.save_for_backward(M, x)
        return ops.bmv(M, x)

    @staticmethod
    def backward(ctx, g):
        M, x = ctx.saved_tensors
        g = g.contiguous()
        dM = ops.bger(g, x) if ctx.needs_input_grad[0] else None
        dx = ops.bmv_t(M, g) if ctx.needs_input_grad[1] else None
        return dM, dx
