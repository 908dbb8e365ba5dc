"""Stage II above the LDS-resident solve's limit (N > 36736, VERDICT r03 "missing" 2: torch.lu has no
size limit, models/lu.py:31-35).

Two forms take over there (csrc/lu.hip): the factorization applies each 128-column block's composed
interchanges to the columns right of the block in a pass of their own and runs the trailing update
without gathered loads (its row tables live in LDS, sized for N <= 36736), and the solve keeps x in
HBM (per 64-row block: one launch for the diagonal triangle, one streaming launch for the rest of
the vector).  The IADMM_LU_FORCE_HBM flag (iadmm_lu_factor_ex / iadmm_lu_solve_ex) sends every size
through both forms, so they are pinned against
the LDS-resident forms at sizes that have both:

* factor: the same arithmetic in the same order, only the interchanges move elsewhere -> the factors
  and pivots must be bit for bit those of the gathered form (both with rank-128 blocks,
  IADMM_LU_RANK128: the paired-block default exists only in the gathered form);
* solve: another summation order -> its distance to the fp64 solution within 2x the LDS-resident
  solve's own distance (+ 1e-6 relative: a random Gaussian matrix's condition number reaches 1e4 and
  more, so both are ~cond x eps away from it; N = 1101 measured 5e-5 between the two), and the
  backward error <= 1e-6 like test_stage2_gpu.py;

then N = 36800 (just past the limit) with a planted permutation built on the device in fp64
(test_stage2_gpu.test_lu_recovers_planted_permutation's construction): partial pivoting must find
exactly the planted rows, the factors must equal L and U to fp32 accuracy, and the solve of
b = A x_true must return x_true to fp32 accuracy (cond ~5)."""
import pytest
import torch

import iadmm_path  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _factor_solve(K, b, force):
    from iadmm import ops
    # (rank-128 blocks on both sides: the paired-block default needs the gathered form, N <= 2048)
    flags = (ops.LU_FORCE_HBM if force else 0) | ops.LU_RANK128
    LU, piv, info = ops.lu_factor(K.clone(), flags=flags)
    x = ops.lu_solve(LU, piv, b, flags=flags & ops.LU_FORCE_HBM)
    torch.cuda.synchronize()
    return LU, piv, info, x


# 130 / 1101: N % 4 != 0 (scalar accesses, partial strips); 2000: the bench's N, several blocks
@pytest.mark.parametrize("N,B", [(130, 2), (1101, 1), (2000, 2)])
def test_hbm_forms_match_lds_forms(N, B):
    g = torch.Generator().manual_seed(N + 7)
    K = torch.randn(B, N, N, generator=g).cuda()
    K[:, 0, 0] = 0.0  # a row interchange at the first step
    b = torch.randn(B, N, generator=g).cuda()
    LU0, piv0, info0, x0 = _factor_solve(K, b, force=False)
    LU1, piv1, info1, x1 = _factor_solve(K, b, force=True)
    assert int(info0.max()) == 0 and int(info1.max()) == 0
    assert torch.equal(piv0, piv1)
    assert torch.equal(LU0.view(torch.int32), LU1.view(torch.int32)), "interchange pass changed the factors"
    Kd = K.double()
    x64 = torch.linalg.solve(Kd, b.double())
    e0 = (x0.double() - x64).norm(dim=1) / x64.norm(dim=1)
    e1 = (x1.double() - x64).norm(dim=1) / x64.norm(dim=1)
    r = torch.bmm(Kd, x1.double().unsqueeze(-1)).squeeze(-1) - b.double()
    berr = float((r.norm(dim=1) / (Kd.flatten(1).norm(dim=1) * x1.double().norm(dim=1))).max())
    print(f"[lu hbm N={N} B={B}] forward error HBM solve {float(e1.max()):.2e}, LDS solve {float(e0.max()):.2e}, "
          f"backward error {berr:.2e}")
    assert bool((e1 <= 2 * e0 + 1e-6).all())
    assert berr < 1e-6


def test_lu_above_lds_limit_planted():
    from iadmm import ops
    N = 36800
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(N)
    s = N ** 0.5
    f64 = dict(generator=g, dtype=torch.float64, device=dev)
    L = torch.tril(torch.rand(N, N, **f64) - 0.5, -1) / s
    L.diagonal().fill_(1.0)
    U = torch.triu(torch.randn(N, N, **f64), 1) / s
    sign = torch.where(torch.rand(N, **f64) < 0.5, -1.0, 1.0)
    U.diagonal().copy_((1.0 + torch.rand(N, **f64)) * sign)
    perm = torch.randperm(N, generator=g, device=dev)
    A = (L @ U)[torch.argsort(perm)]              # row perm[i] of A is row i of L U
    packed = torch.tril(L, -1) + U
    del L, U
    xt = torch.randn(N, **f64)
    b = (A @ xt).float().unsqueeze(0)
    Af = A.float().unsqueeze(0).contiguous()
    del A
    torch.cuda.empty_cache()
    LU, piv, info = ops.lu_factor(Af)
    x = ops.lu_solve(LU, piv, b)
    torch.cuda.synchronize()
    assert int(info[0]) == 0
    rows = list(range(N))
    for i, p in enumerate(piv[0].cpu().tolist()):  # the 1-based swap sequence as a permutation
        rows[i], rows[p - 1] = rows[p - 1], rows[i]
    assert rows == perm.cpu().tolist()
    ferr_lu = float((LU[0].double() - packed).norm() / packed.norm())
    ferr_x = float((x[0].double() - xt).norm() / xt.norm())
    print(f"[lu hbm N={N}] factors rel-L2 {ferr_lu:.2e}, solve rel-L2 to x_true {ferr_x:.2e}")
    assert ferr_lu < 1e-5
    assert ferr_x < 1e-5
