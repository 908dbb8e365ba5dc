"""Stage II (models/lu.py) on the GPU: batched LU + solve against the reference's golden Stage-II
iterates and against fp64 solves.

Tolerances: LU solves are compared by backward error ||K x - b|| / (||K|| ||x||) <= 1e-6 (fp32
partial pivoting); the Stage-II iterates vs the golden ones (MKL getrf) rel-L2 <= 1e-4 on x and z
and 1e-3 on the final residuals (the KKT matrix with rho_eq ~ 500 has condition ~1e4, so
forward errors are ~cond x eps)."""
import numpy as np
import pytest
import torch

import iadmm_path  # noqa: F401

pytestmark = pytest.mark.gpu


def rel_l2(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-30))


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


# 16 / 37 / 64: one 64-column block (single-row-slot panels); 100, 130, 257, 1101 (N % 4 != 0:
# scalar trailing-update accesses; 1101 also two 1024-row trailing chunks and 4- and 8-slot
# panels); 400, 2000: several blocks with partial 128-column strips and 64-row steps
# 2049 .. 10000: the 8-column panels on 1024-thread workgroups (N > 2048; 5003: N % 4 != 0;
# 10000 = config 4's N, 10 panel rows per thread at the first panel); 12000 / 12291: the first
# panels exceed the registers' 10240 rows and run from HBM (lu_panel_global_kernel; 12291: N % 4 != 0)
@pytest.mark.parametrize("N,B", [(16, 2), (37, 3), (64, 2), (100, 2), (130, 2), (257, 2), (400, 2), (1101, 1),
                                 (2000, 1), (2049, 2), (2500, 1), (5003, 1), (10000, 1), (12000, 1), (12291, 1)])
def test_lu_factor_solve_backward_error(N, B):
    from iadmm import ops
    g = torch.Generator().manual_seed(N)
    K = torch.randn(B, N, N, generator=g)
    K[:, 0, 0] = 0.0  # forces a row interchange at the first step
    b = torch.randn(B, N, generator=g)
    LU, piv, info = ops.lu_factor(K.cuda().contiguous())
    x = ops.lu_solve(LU, piv, b.cuda())
    assert int(info.max()) == 0
    Kd, xd, bd = K.double(), x.double().cpu(), b.double()
    r = torch.bmm(Kd, xd.unsqueeze(-1)).squeeze(-1) - bd
    berr = r.norm(dim=1) / (Kd.flatten(1).norm(dim=1) * xd.norm(dim=1))
    assert float(berr.max()) < 1e-6
    assert (piv[:, 0].cpu() != 1).all()
    if N > 2049:
        return
    # LAPACK's 1-based pivot convention: the factors feed torch.linalg.lu_solve unchanged
    # (the two fp32 substitutions differ in summation order, so compare backward errors, not x)
    xt = torch.linalg.lu_solve(LU, piv, b.cuda().unsqueeze(-1)).squeeze(-1).double().cpu()
    rt = torch.bmm(Kd, xt.unsqueeze(-1)).squeeze(-1) - bd
    assert float((rt.norm(dim=1) / (Kd.flatten(1).norm(dim=1) * xt.norm(dim=1))).max()) < 1e-6


# one 64-column block; several (deferred block interchanges).  Larger random matrices have
# near-ties between candidate pivots that fp32 and LAPACK's fp64 resolve differently (N = 2500
# differed), so the large-N pivot logic is pinned by test_lu_recovers_planted_permutation.
@pytest.mark.parametrize("N", [48, 300])
def test_lu_pivots_match_lapack_choice(N):
    """Same pivot sequence as partial pivoting with first-max tie-breaking (LAPACK i?amax)."""
    from iadmm import ops
    g = torch.Generator().manual_seed(7)
    K = torch.randn(2, N, N, generator=g)
    LU, piv, _ = ops.lu_factor(K.cuda().contiguous())
    threads = torch.get_num_threads()
    torch.set_num_threads(1)  # this torch build's multi-threaded MKL LASWP can hang
    try:
        lu_ref, ref = torch.linalg.lu_factor(K.double())
    finally:
        torch.set_num_threads(threads)
    assert torch.equal(piv.cpu().long(), ref.long())
    # same pivots -> the same factors up to fp32 rounding growth (L and U packed like LAPACK's)
    assert rel_l2(LU, lu_ref) < 1e-5


@pytest.mark.parametrize("N", [300, 2000, 2500, 5003, 10500])
def test_lu_recovers_planted_permutation(N):
    """A = P0 L U with well-conditioned unit-lower L and upper U (off-diagonals scaled by
    1/sqrt(N), |diag U| in [1, 2]; cond ~2 and ~5): at every step the row of L's diagonal beats
    every other candidate by > sqrt(N), so partial pivoting must choose exactly P0 (no
    near-ties, unlike random matrices) and the factors must equal L and U to fp32 accuracy (the LU
    of P0^T A is unique; LAPACK sgetrf gives ~1e-7).  Covers both panel shapes (16-wide <= 2048 <
    8-wide; 10500: the panels with more than 10240 rows, k0 < 260, from HBM, the rest in registers)."""
    from iadmm import ops
    g = torch.Generator().manual_seed(N)
    s = N ** 0.5
    f64 = dict(generator=g, dtype=torch.float64)
    L = torch.eye(N, dtype=torch.float64) + torch.tril(torch.rand(N, N, **f64) - 0.5, -1) / s
    U = torch.triu(torch.randn(N, N, **f64), 1) / s
    U += torch.diag((1.0 + torch.rand(N, **f64)) * torch.where(torch.rand(N, generator=g) < 0.5, -1.0, 1.0).double())
    perm = torch.randperm(N, generator=g)
    A = (L @ U)[torch.argsort(perm)]          # row perm[i] of A is row i of L U
    LU, piv, info = ops.lu_factor(A.float().unsqueeze(0).cuda().contiguous())
    assert int(info[0]) == 0
    rows = list(range(N))
    for i, p in enumerate(piv[0].cpu().tolist()):  # the 1-based swap sequence as a permutation
        rows[i], rows[p - 1] = rows[p - 1], rows[i]
    assert rows == perm.tolist()
    packed = torch.tril(L, -1) + U
    assert rel_l2(LU[0], packed) < 1e-5


def test_stage2_chunks_equal_full_batch():
    """solver.stage2 factoring the batch in chunks (config 4's K does not fit at once) gives the
    full-batch result bit for bit, histories included (every kernel works per instance)."""
    from iadmm import data, solver
    n, mi, me, B = 60, 20, 12, 5
    d = data.make_qp_batch(n, mi, me, B, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(B, n, device="cuda", generator=g)
    y = torch.randn(B, mi + me, device="cuda", generator=g)
    z = torch.randn(B, mi + me, device="cuda", generator=g)
    rho = torch.full((B, mi + me), 0.5, device="cuda")
    rho[:, mi:] = 500.0
    args = (d["Q"], d["p"].reshape(B, n).contiguous(), d["A0"], d["zl"].reshape(B, -1).contiguous(),
            d["zu"].reshape(B, -1).contiguous(), rho, x, y, z, 6e-6, 4)
    seen = []
    full = solver.stage2(*args, history=True)
    part = solver.stage2(*args, history=True, chunk=2, iter_hook=lambda t, xc, yc, zc, sl: seen.append((t, sl)))
    assert full["chunk"] == B and part["chunk"] == 2
    for k in ("x", "y", "z", "xv", "hist_obj", "hist_ls_res", "hist_primal", "hist_dual"):
        assert torch.equal(full[k], part[k]), k
    assert [sl for t, sl in seen if t == 0] == [slice(0, 2), slice(2, 4), slice(4, 5)]
    assert float(full["hist_ls_res"].max()) < 1e-2 * float(full["hist_primal"].abs().max() + 1)


def test_lu_singular_reports_info():
    from iadmm import ops
    K = torch.randn(1, 32, 32)
    K[0, :, 5] = 0.0
    _, _, info = ops.lu_factor(K.cuda().contiguous())
    assert int(info[0]) > 0


def test_stage2_golden(golden):
    from models.lu import LU
    name, g = golden
    n, mi, me, h, T, B, scaling, stage2 = (int(v) for v in g["meta"])
    if not stage2:
        pytest.skip("no Stage II in this fixture")
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    x, y, z, xv, rv = (dev(g[k]) for k in ("fin_x", "fin_y", "fin_z", "fin_xv", "fin_rhovec"))
    kw = {k: dev(g["in_" + k]) for k in ("Q", "p", "A0", "zl", "zu")}
    model = LU("cuda")
    A_t = lu = piv = None
    with torch.no_grad():
        for it in range(stage2):
            x, y, z, xv, A_t, bt, lu, piv = model(rv, x, y, z, xv, float(g["sigma"]), A_t, lu, piv,
                                                  lb=None, ub=None, **kw)
            assert rel_l2(x, g["s2_x"][it]) < 1e-4, (name, it)
            assert rel_l2(z, g["s2_z"][it]) < 1e-4, (name, it)
        import utils
        pr, du, _ = utils.primal_dual_loss(x, y, z, kw["Q"], kw["p"], kw["A0"])
    np.testing.assert_allclose(pr.reshape(-1).cpu().numpy(), g["s2_primal"], rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(du.reshape(-1).cpu().numpy(), g["s2_dual"], rtol=1e-3, atol=1e-5)
    # the returned A_tild is K with the same rho (main.py:1072 ls_res)
    from oracle import iadmm_oracle as orc
    K = orc.kkt_matrix(torch.from_numpy(g["in_Q"]), torch.from_numpy(g["in_A0"]), float(g["sigma"]),
                       torch.from_numpy(g["fin_rhovec"]))
    assert rel_l2(A_t.dense(), K) < 1e-7


# n, m multiples of 4 -> the 16-B row-band kernel (n % 32 != 0: a band straddling the Q / A0 rows;
# m > 256: several LDS chunks of the A0^T block); otherwise the 64 x 64 tile kernel
@pytest.mark.parametrize("n,m", [(1000, 1000), (100, 300), (36, 20), (64, 0), (37, 15), (24, 12), (40, 6)])
def test_kkt_assemble_bitwise(n, m):
    """iadmm_kkt_assemble builds exactly the reference's K (models/lu.py:27-28 / models/lstm.py:67-68:
    copies, one sigma add per diagonal, -(1/rho) on the lower-right diagonal, -0 elsewhere)."""
    from iadmm import ops
    from oracle import iadmm_oracle as orc
    B = 2
    g = torch.Generator().manual_seed(n + m)
    Q, A0 = torch.randn(B, n, n, generator=g), torch.randn(B, m, n, generator=g)
    rho = torch.rand(B, m, generator=g) + 0.05
    K = ops.kkt_assemble(Q.cuda(), A0.cuda(), 6e-6, None, 0, rho_rows=rho.cuda())
    ref = orc.kkt_matrix(Q, A0, 6e-6, rho.unsqueeze(-1))
    assert torch.equal(K.cpu(), ref)
    assert torch.equal(torch.signbit(K.cpu()), torch.signbit(ref))


@pytest.mark.parametrize("N,B", [(2000, 3), (1024, 2), (516, 2), (1024, 512)])
def test_paired_blocks_match_rank128_form(N, B):
    """Paired blocks (r05, the default for N <= 2048, csrc/lu.hip lu_trail256_kernel: one rank-256 update
    of the columns right of every two 128-column blocks, the pair's interchanges composed into one gather)
    against the rank-128-per-block form (IADMM_LU_RANK128) on the same KKT-like matrices: a different summation
    order, so not bitwise -- the backward errors ||PLU - K|| / ||K|| stay within
    1.5x of each other, and both solves land within 2x of each other's distance to the fp64 solution.
    N = 516: an odd block count with a partial last block (the last pair is a single block).
    B = 512: the paired default then splits the batch over the context's two streams -- checked
    against rank-128 as above and bitwise against the same factorization on one stream."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from iadmm import ops
    g = torch.Generator().manual_seed(N + 31)
    n = N // 2
    Q = torch.diag_embed(torch.rand(B, n, generator=g)) + 6e-6 * torch.eye(n)
    A0 = torch.randn(B, N - n, n, generator=g)
    K = torch.zeros(B, N, N)
    K[:, :n, :n] = Q
    K[:, :n, n:] = A0.transpose(1, 2)
    K[:, n:, :n] = A0
    K[:, n:, n:] = -torch.diag_embed(torch.where(torch.arange(N - n) < (N - n) // 2, 2.0, 0.002)).expand(B, -1, -1)
    K = K.cuda()
    b = torch.randn(B, N, generator=g).cuda()
    res = {}
    for name, fl in (("paired", 0), ("rank128", ops.LU_RANK128)):
        LU, piv, info = ops.lu_factor(K.clone(), flags=fl)
        x = ops.lu_solve(LU, piv, b)
        torch.cuda.synchronize()
        assert int(info.max()) == 0
        Kd = K.double()
        P, L, U = torch.lu_unpack(LU.double(), piv)
        berr = ((P @ (L @ U) - Kd).flatten(1).norm(dim=1) / Kd.flatten(1).norm(dim=1))
        x64 = torch.linalg.solve(Kd, b.double())
        ferr = (x.double() - x64).norm(dim=1) / x64.norm(dim=1)
        res[name] = (piv, berr, ferr)
        if name == "paired" and B >= 512:
            LU1, piv1, _ = ops.lu_factor(K.clone(), flags=fl, lookahead=False)
            torch.cuda.synchronize()
            assert torch.equal(LU1, LU) and torch.equal(piv1, piv), "batch split differs from one stream"
            del LU1
        del LU
    print(f"[paired N={N}] backward error paired {res['paired'][1].tolist()} rank-128 {res['rank128'][1].tolist()}; "
          f"forward error paired {res['paired'][2].tolist()} rank-128 {res['rank128'][2].tolist()}")
    # (no pivot comparison: a different summation order breaks near-ties in the pivot search, and one
    # different pivot changes every later one -- measured 88 % agreement at N = 2000 with equal
    # backward errors; the factorisation is pinned by its backward error instead)
    assert bool((res["paired"][1] <= 1.5 * res["rank128"][1]).all())
    assert bool((res["paired"][2] <= 2 * res["rank128"][2] + 1e-6).all())
