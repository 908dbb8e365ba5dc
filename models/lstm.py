"""Drop-in ``models.lstm.LSTM`` (reference: models/lstm.py:6-96), HIP-backed.

Same constructor, parameter names/shapes/initialisation order (so ``load_state_dict`` of a
reference ``.pth`` works, main.py:618), same ``forward`` signature and return tuple.  One call
runs three gfx950 kernels through libiadmm.so:
  iadmm_kkt_resgrad   g = K^T(K xv - b~) with K never materialised   (lstm.py:67-72)
  iadmm_lstm_cell_fwd 4 gate GEMMs on fp32 MFMA + fused cell update  (lstm.py:74-80)
  iadmm_admm_update   xv / x / z / y updates                         (lstm.py:80-94)
``A_tild`` comes back as a lazy :class:`iadmm.kktop.KKTOperator` (``torch.bmm(A_tild, xv)``
works; ``.dense()`` materialises K).  Outputs are fresh tensors (functional semantics): the
caller may keep its inputs.  Under grad mode the call goes through
:class:`iadmm.autograd.IterationFn`, whose backward is a set of HIP kernels (training).
"""
import torch
import torch.nn as nn

import iadmm_path  # noqa: F401
from iadmm import ops
from iadmm.kktop import KKTOperator
from iadmm.autograd import IterationFn, window_grads_for
from iadmm.solver import PARAM_NAMES, PackedWeights, param_dict

_GATES = ("i", "f", "o", "u")


class LSTM(nn.Module):
    RHO_EQ_OVER_RHO_INEQ = 1e03  # fixed in the kernels (models/lstm.py:18)

    def __init__(self, num_constr, input_dim, hidden_dim, length, device):
        super().__init__()
        if input_dim != 2:
            raise ValueError("the I-ADMM-LSTM cell consumes [xv, K^T(K xv - b)]: input_dim must be 2")
        self.num_constr = num_constr
        self.input_dim = input_dim
        self.hidden_dim = hidden_dim
        self.length = length
        self.device = device

        def normal(*shape):
            return nn.Parameter(torch.normal(mean=0, std=0.01, size=shape, device=device))

        def zeros(*shape):
            return nn.Parameter(torch.zeros(shape, device=device, dtype=torch.float32))

        # draw order = reference order (i, f, o, u gates; W, U, b each), then W_h, b_h, rho, alpha
        for gname in _GATES:
            setattr(self, "W_" + gname, normal(input_dim, hidden_dim))
            setattr(self, "U_" + gname, normal(hidden_dim, hidden_dim))
            setattr(self, "b_" + gname, zeros(hidden_dim))
        self.W_h = normal(hidden_dim, 1)
        self.b_h = zeros(1)
        self.rho = normal(length, 1)
        self.alpha = normal(length, 1)
        self._packed = PackedWeights()

    def name(self):
        return "lstm"

    def forward(self, t, num_ineq, num_eq, x, y, z, xv, sigma, H_t, C_t, **kwargs):
        Q, p, A0, zl, zu = (kwargs[k] for k in ("Q", "p", "A0", "zl", "zu"))
        B, n = x.shape[0], x.shape[1]
        m = y.shape[1]
        if num_ineq + num_eq != m:
            raise ValueError(f"num_ineq + num_eq = {num_ineq + num_eq} != {m} constraint rows")
        if t >= self.length:
            raise IndexError(f"iteration {t} >= model length {self.length} (models/lstm.py:60)")
        N, h = n + m, self.hidden_dim
        c = lambda a: a.detach().float().contiguous()  # noqa: E731
        Q, A0 = c(Q), c(A0)
        pv, xv_, xv2 = c(p).reshape(B, n), c(x).reshape(B, n), c(xv).reshape(B, N)
        yv, zvv = c(y).reshape(B, m), c(z).reshape(B, m)
        zlv, zuv = c(zl).reshape(B, m), c(zu).reshape(B, m)
        params = param_dict(self)
        if torch.is_grad_enabled() and (any(v.requires_grad for v in params.values()) or any(
                isinstance(v, torch.Tensor) and v.requires_grad for v in (x, y, z, xv, H_t, C_t))):
            return self._forward_autograd(t, num_ineq, sigma, x, y, z, xv, H_t, C_t, Q, pv, A0, zlv, zuv, params)

        scal = ops.schedule(c(self.rho), c(self.alpha), t)
        btild = ops.empty(B, N, like=Q)
        rho_vec = ops.empty(B, m, like=Q)
        g = ops.kkt_resgrad(Q, A0, pv, xv_, yv, zvv, xv2, float(sigma), scal, num_ineq,
                            btild=btild, rho_vec=rho_vec)
        Upk, Wx = self._packed.get(params, h)
        Hn, Cn, part = ops.lstm_cell(c(H_t), c(C_t), xv2, g, Upk, Wx)
        xvo, xo, yo, zo = ops.admm_update(n, m, num_ineq, part, c(self.b_h), xv2, xv_, yv, zvv, zlv, zuv, scal)
        A_tild = KKTOperator(Q, A0, sigma, scal, num_ineq)
        return (xo.unsqueeze(-1), yo.unsqueeze(-1), zo.unsqueeze(-1), xvo.unsqueeze(-1), Hn, Cn,
                A_tild, btild.unsqueeze(-1), rho_vec.unsqueeze(-1))

    def _forward_autograd(self, t, num_ineq, sigma, x, y, z, xv, H_t, C_t, Q, pv, A0, zlv, zuv, params):
        """Training path: the same kernels wrapped in iadmm.autograd.IterationFn, whose backward
        runs the HIP backward kernels (TBPTT through main.py:336-350)."""
        B, n = x.shape[0], x.shape[1]
        m = y.shape[1]
        N = n + m
        flat = lambda a, k: a.float().reshape(B, k).contiguous()  # noqa: E731 (keeps autograd)
        Hc = H_t.float().contiguous()
        plist = [params[k] for k in PARAM_NAMES]
        acc, owner = window_grads_for(Hc, plist)  # the window's shared parameter-gradient sums (r06)
        meta = (int(t), int(num_ineq), float(sigma), (Q, pv, A0, zlv, zuv), self._packed, acc, owner)
        xo, yo, zo, xvo, Hn, Cn, btild, rho_vec = IterationFn.apply(
            meta, flat(x, n), flat(y, m), flat(z, m), flat(xv, N), Hc, C_t.float().contiguous(), *plist)
        A_tild = KKTOperator(Q, A0, sigma, ops.schedule(self.rho.detach().contiguous(),
                                                        self.alpha.detach().contiguous(), t), num_ineq)
        return (xo.unsqueeze(-1), yo.unsqueeze(-1), zo.unsqueeze(-1), xvo.unsqueeze(-1), Hn, Cn,
                A_tild, btild.unsqueeze(-1), rho_vec.unsqueeze(-1))
