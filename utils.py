"""Drop-in ``utils`` (reference: utils.py:7-78): checkpoint policy + metrics.

Metrics on device tensors run on gfx950 kernels (iadmm_metrics, iadmm_bmv); ``lb_dist`` /
``ub_dist`` are single elementwise clamps.  ``EarlyStopping`` keeps the reference policy and its
state-dict checkpoint format.
"""
import torch
import numpy as np

import iadmm_path  # noqa: F401
from iadmm import ops


class EarlyStopping(object):
    """Saves ``model.state_dict()`` when every violation <= tol and the loss improved
    (utils.py:7-50); stops after ``patience`` epochs without a save."""

    def __init__(self, save_path, patience=10):
        self.filename = save_path
        self.patience = patience
        self.counter = 0
        self.best_loss = None
        self.early_stop = False

    def _bad_epoch(self):
        self.counter += 1
        print(f'EarlyStopping counter: {self.counter} out of {self.patience}')

    def step(self, loss, model, mode, tol, *args):
        if not all(vio <= tol for vio in args):
            self._bad_epoch()
        elif self.best_loss is None:
            self.best_loss = loss
            self.save_checkpoint(model)
            self.counter = 0
        elif mode in ("min", "max"):
            better = loss <= self.best_loss if mode == "min" else loss >= self.best_loss
            if better:
                self.save_checkpoint(model)
                self.best_loss = (np.min if mode == "min" else np.max)((loss, self.best_loss))
                self.counter = 0
            else:
                self._bad_epoch()
        if self.counter >= self.patience:
            self.early_stop = True
        return self.early_stop

    def save_checkpoint(self, model):
        torch.save(model.state_dict(), self.filename)

    def load_checkpoint(self, model):
        model.load_state_dict(torch.load(self.filename, weights_only=True))


def _flat(a):
    return a.detach().float().reshape(a.shape[0], -1).contiguous()


def _wants_grad(*ts):
    return torch.is_grad_enabled() and any(isinstance(t, torch.Tensor) and t.requires_grad for t in ts)


def _f32(a):
    """fp32 contiguous view that keeps the autograd graph (the Functions below get differentiable
    inputs; their backward kernels compute in fp32 like the forward)."""
    return a.float().contiguous()


def obj_fn(x, Q, p):
    """1/2 x^T Q x + p^T x, [B,1,1] (utils.py:53-54).  Differentiable in x, Q, p
    (iadmm.autograd.ObjFn: backward on iadmm_bmv / iadmm_bmv_t / iadmm_bger)."""
    B, n = x.shape[0], x.shape[1]
    if _wants_grad(x, Q, p):
        from iadmm.autograd import ObjFn
        return ObjFn.apply(_f32(x.reshape(B, n)), _f32(Q), _f32(p.reshape(B, n))).reshape(B, 1, 1)
    zeros = x.new_zeros(B, 0)
    obj, _, _ = ops.metrics(Q.detach().float().contiguous(), _flat(p), Q.new_zeros(B, 0, n), _flat(x), zeros, zeros)
    return obj.reshape(B, 1, 1)


def ineq_dist(x, G, c):
    """max(G x - c, 0), [B,mi,1] (utils.py:56-57).  Differentiable in x, G, c (IneqDistFn)."""
    if _wants_grad(x, G, c):
        from iadmm.autograd import IneqDistFn
        B = x.shape[0]
        return IneqDistFn.apply(_f32(x.reshape(B, -1)), _f32(G), _f32(c.reshape(B, -1))).unsqueeze(-1)
    return ops.bmv(G.detach().float().contiguous(), _flat(x), _flat(c), ops.BMV_POS_EXCESS).unsqueeze(-1)


def eq_dist(x, A, b):
    """|b - A x|, [B,me,1] (utils.py:59-60).  Differentiable in x, A, b (EqDistFn)."""
    if _wants_grad(x, A, b):
        from iadmm.autograd import EqDistFn
        B = x.shape[0]
        return EqDistFn.apply(_f32(x.reshape(B, -1)), _f32(A), _f32(b.reshape(B, -1))).unsqueeze(-1)
    return ops.bmv(A.detach().float().contiguous(), _flat(x), _flat(b), ops.BMV_ABS_GAP).unsqueeze(-1)


def lb_dist(x, lb):
    """utils.py:62-63."""
    return torch.clamp(lb - x, 0)


def ub_dist(x, ub):
    """utils.py:65-66."""
    return torch.clamp(x - ub, 0)


def primal_dual_loss(x, y, z, Q, p, A0):
    """(||A0 x - z||, ||Q x + p + A0^T y||, sum), each [B,1,1] (utils.py:68-71).  Differentiable
    in x, y, z (the training loss, main.py:346) and in the data through iadmm.autograd.LossFn."""
    B = x.shape[0]
    if _wants_grad(x, y, z, Q, p, A0):
        from iadmm.autograd import LossFn
        pr, du = LossFn.apply(_f32(x.reshape(B, -1)), _f32(y.reshape(B, -1)), _f32(z.reshape(B, -1)), _f32(Q),
                              _f32(p.reshape(B, -1)), _f32(A0))
        pr, du = pr.reshape(B, 1, 1), du.reshape(B, 1, 1)
        return pr, du, pr + du
    _, pr, du = ops.metrics(Q.detach().float().contiguous(), _flat(p), A0.detach().float().contiguous(),
                            _flat(x), _flat(y), _flat(z))
    pr, du = pr.reshape(B, 1, 1), du.reshape(B, 1, 1)
    return pr, du, pr + du


def aug_lagr(x, z, y, Q, p, A0, rho_vec):
    """utils.py:74-78, including the reference's ``Q p`` (not ``Q x``) in the quadratic term;
    only used by commented-out analysis code in the reference.  Under grad the two matvecs run as
    iadmm.autograd.BmvFn (HIP forward and backward) and the rest is elementwise."""
    B = x.shape[0]
    if _wants_grad(x, z, y, Q, p, A0, rho_vec):
        from iadmm.autograd import BmvFn
        xf, zf, yf, pf, rf = (_f32(t.reshape(B, -1)) for t in (x, z, y, p, rho_vec))
        Qp = BmvFn.apply(_f32(Q), pf)
        r = BmvFn.apply(_f32(A0), xf) - zf
    else:
        xf, zf, yf, pf, rf = (_flat(t) for t in (x, z, y, p, rho_vec))
        Qp = ops.bmv(Q.detach().float().contiguous(), pf)
        r = ops.bmv(A0.detach().float().contiguous(), xf) - zf
    fx = 0.5 * (xf * Qp).sum(1) + (pf * xf).sum(1)
    dual_item = (yf * r).sum(1)
    aug_item = 0.5 * (r * (rf * r)).sum(1)
    return (fx + dual_item + aug_item).reshape(-1, 1, 1)
