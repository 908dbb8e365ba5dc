"""K = 100 parity at the headline instance shape (BASELINE config 2: n=1000, m=500+500, h=800).

The HIP solve (Ruiz -> 100 Stage-I iterations -> unscale) of the bench's first two instances
against the CPU oracle run in fp32 AND fp64 on the same instances and weights, every iteration
(tests/k100_envelope.py): the GPU's distance to the fp64 trajectory must stay
within 2x the fp32 oracle's own distance to it (+ 1e-7 relative) for x, y, z, the residual
vectors r_p = A0x - z, r_d = Qx + p + A0^T y and the reported primal / dual metrics.  r04's fixed
1e-4 relative bound on the residual histories is gone: it failed for a better-trained save
(epoch 42: 6.5e-4) while x, y, z stayed close, and a fixed bound lets the choice of weights decide
the verdict.  Weight sets:

* ``trained`` -- checkpoints/QP_1000_500_500_100_800.pth (the reference recipe, checkpoints/README.md);
* every other save of that run kept under checkpoints/candidates/ (``e30``, ``e55``, ...);
* ``random-init`` -- the reference's initialisation (the solve diverges at this shape: primal
  residual ~1e4 after 100 iterations; the envelope holds the same way).
"""
import glob
import os

import pytest
import torch

import iadmm_path  # noqa: F401
import k100_envelope as env
from oracle import iadmm_oracle as orc

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CKPT = os.path.join(REPO, "checkpoints", "QP_1000_500_500_100_800.pth")
CANDIDATES = {os.path.basename(f)[len("QP_1000_500_500_100_800_"):-4]: f
              for f in sorted(glob.glob(os.path.join(REPO, "checkpoints", "candidates", "QP_1000_500_500_100_800_*.pth")))}
N_VAR, MI, ME, H, T, B = 1000, 500, 500, 800, 100, 2
SIGMA = 6e-6
TAGS = ["trained", *CANDIDATES, "random-init"]
# the optional f16x3 cell: its gate GEMM carries 22 significant bits, not 24 -- 4x the unit
# roundoff of the fp32 path -- so its envelope is 4 x the fp32 factor (stated before measuring)
F16X3_FACTOR = 4 * env.FACTOR


def rel_l2_rows(a, b):
    a = torch.as_tensor(a).double().cpu().reshape(B, -1)
    b = torch.as_tensor(b).double().cpu().reshape(B, -1)
    return float(((a - b).norm(dim=1) / b.norm(dim=1).clamp_min(1e-30)).max())


@pytest.fixture(scope="module")
def batch():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from iadmm import data
    return data.make_qp_batch(N_VAR, MI, ME, B, first_index=0, device="cuda")


def weights(tag):
    from iadmm import data
    from iadmm.solver import PARAM_NAMES
    if tag == "random-init":
        return data.init_lstm_params(H, T, device="cuda")
    f = CKPT if tag == "trained" else CANDIDATES[tag]
    if not os.path.exists(f):
        pytest.skip(f"no checkpoint at {f}")
    sd = torch.load(f, map_location="cuda", weights_only=True)
    return {k: sd[k].float().contiguous() for k in PARAM_NAMES}


_RUNS = {}


def k100_run(batch, tag):
    """(GPU solve, fp32 oracle, fp64 oracle) of the two instances for one weight set, computed once
    per module (the Stage-II test below starts from the fp32 oracle's end state)."""
    if tag not in _RUNS:
        params = weights(tag)
        cpu = {k: v.cpu() for k, v in batch.items()}
        out = env.gpu_run(params, batch, MI, ME, T, SIGMA)
        r32 = env.oracle_run(params, cpu, MI, ME, T, SIGMA, H, torch.float32)
        r64 = env.oracle_run(params, cpu, MI, ME, T, SIGMA, H, torch.float64)
        _RUNS[tag] = (out, r32, r64)
    return _RUNS[tag]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("tag", TAGS)
def test_k100_envelope(batch, tag):
    out, ref, r64 = k100_run(batch, tag)
    cpu = {k: v.cpu() for k, v in batch.items()}
    fails, _ = env.check(out, ref, r64, cpu, tag)
    # for the record: the r04 statistics against the fp32 oracle (no longer a bound)
    err = {k: rel_l2_rows(out[k], ref[k]) for k in ("x", "y", "z")}
    hist = {}
    for k in ("primal", "dual"):
        a = out["hist_" + k].double().cpu()
        hist[k] = float(((a - ref["hist_" + k].double()).abs() / ref["hist_" + k].double().abs().clamp_min(1e-6)).max())
        hist[k + "64"] = float(((ref["hist_" + k].double() - r64["hist_" + k]).abs() / r64["hist_" + k].abs()).max())
    print(f"[k100 {tag}] vs fp32 oracle: rel-L2 x {err['x']:.2e} y {err['y']:.2e} z {err['z']:.2e} | hist max rel "
          f"primal {hist['primal']:.2e} dual {hist['dual']:.2e} (fp32 oracle vs fp64: {hist['primal64']:.2e} / "
          f"{hist['dual64']:.2e}) | final primal {r64['primal'].tolist()} dual {r64['dual'].tolist()}")
    assert not fails, fails[:4]
    if tag != "random-init":  # a trained save's point: the residuals fall over K
        pr = r64["hist_primal"].mean(1)
        du = r64["hist_dual"].mean(1)
        assert float(pr[-1] + du[-1]) < float((pr + du)[:10].max())


@pytest.mark.timeout(900)
def test_k100_f16x3_envelope(batch):
    """The optional split-precision cell (precision="f16x3", csrc/lstm_f16x3.hip) over the whole
    K = 100 solve, against the same fp32 / fp64 oracle runs, under the envelope with F16X3_FACTOR
    (its 22-bit gate GEMM: 4x the fp32 path's unit roundoff)."""
    from iadmm import solver
    out32, ref, r64 = k100_run(batch, "trained")
    tr = {"x": [], "y": [], "z": []}

    def hook(t, ux, uy, uz):
        for k, v in zip("xyz", (ux, uy, uz)):
            tr[k].append(v.clone())

    d = batch
    with torch.no_grad():
        out = solver.solve(weights("trained"), d["Q"], d["p"], d["A0"], d["zl"], d["zu"], MI, ME, T, SIGMA,
                           history=True, precision="f16x3", iter_hook=hook)
    for k in tr:
        out["trace_" + k] = torch.stack(tr[k]).double().cpu()
    cpu = {k: v.cpu() for k, v in batch.items()}
    fails, _ = env.check(out, ref, r64, cpu, "f16x3", verbose=False, factor=F16X3_FACTOR)
    line = [f"{k} {rel_l2_rows(out[k], r64[k]):.2e} (f32 {rel_l2_rows(out32[k], r64[k]):.2e})" for k in "xyz"]
    print("[k100 f16x3 vs fp64] " + " | ".join(line))
    assert not fails, fails[:4]


STAGE2_ITERS = 20  # feas_rest_num of the bench's Stage-II record


@pytest.mark.timeout(600)
def test_stage2_after_k100_vs_oracle(batch):
    """Stage II (models/lu.py, main.py:1035-1077) at the config-2 shape, N = 2000: from the
    oracle's Stage-I end state of the trained K = 100 run (unscaled x, y, z, xv; the last scaled
    rho_vec), 20 exact iterations through the drop-in LU module on the GPU (HIP LU factor + solves)
    and through oracle.lu_iteration (LAPACK getrf/getrs, one thread) in fp32 and fp64.  Bound:
    tests/stage2_envelope.py (per iteration: x, y, z and the residual vectors within 2x the fp32
    oracle's distance to fp64, the reported primal/dual metrics within 2x its residual-vector
    distance); the factorisation backward errors are printed and compared with MKL's."""
    import stage2_envelope
    _, ref, _ = k100_run(batch, "trained")
    cpu = {k: v.cpu() for k, v in batch.items()}
    st0 = {k: ref[k].clone() for k in ("x", "y", "z", "xv", "rho_vec")}
    rows, fails, berr, r32 = stage2_envelope.run(st0, cpu, STAGE2_ITERS, "N=2000")
    assert not fails, fails[:4]
    for b in berr:
        assert b["hip"]["berr"] <= 1.5 * b["mkl"]["berr"], b  # r05 two-level U12 (r04: 2.0x, measured 1.33-1.8x)
    # the bench's observation (primal falls under Stage II) is the oracle's too
    pr0, _, _ = orc.primal_dual(st0["x"], st0["y"], st0["z"], cpu["Q"], cpu["p"], cpu["A0"])
    prK, _, _ = orc.primal_dual(*(r32[-1][k].float() for k in ("x", "y", "z")), cpu["Q"], cpu["p"], cpu["A0"])
    assert float(prK.mean()) < float(pr0.mean())
