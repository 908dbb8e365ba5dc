"""bench.py / bench_train.py contract on the GPU: the one-line JSON of a single-GPU run, and the
N > 1 code path (instance sharding, barriers, max-over-ranks timing, gradient all-reduce)
rehearsed with two ranks sharing cuda:0 over gloo (IADMM_SHARED_GPU=1; RCCL refuses two ranks on
one device).  Small shapes; the full-size numbers come from the round-end bench runs."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--num_var", "64", "--num_ineq", "32", "--num_eq", "32", "--hidden_dim", "64", "--outer_T", "3"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, nproc=1, timeout=600, shared=True, extra_env=None, launcher=False):
    """Run a bench script; under torch.distributed.run when nproc > 1 (or launcher=True), with the
    ranks sharing cuda:0 over gloo when ``shared``, one GPU per rank over RCCL otherwise."""
    env = dict(os.environ)
    env.update(extra_env or {})
    if nproc > 1 and shared:
        env["IADMM_SHARED_GPU"] = "1"
    if nproc > 1 or launcher:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] + args + ["--gpus", str(nproc)]
    else:
        cmd = [sys.executable] + args
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_bench_single_gpu_contract():
    r = _run(["bench.py", "--batch", "8", "--steps", "2", "--warmup", "1", "--cpu-sample", "2"] + SMALL)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in r, k
    assert r["n_gpus"] == 1 and r["steps"] == 2 and r["warmup"] == 1 and r["higher_is_better"] is True
    assert r["value"] > 0 and r["config"]["global_batch"] == 8
    rf = r["roofline"]
    assert rf["bound"] == "mfma" and rf["unit"] == "TFLOP/s" and rf["launches"] == 2 * 3
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    cb = r["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1 and cb["cpu_model"]
    # the GPU's result on the CPU sample's instances against the oracle's (same instances)
    par = cb["parity"]["random-init"]
    assert par["within_tol"], par
    assert par["x_rel_l2"] <= par["tol"]["x"] and par["primal_max_rel"] <= par["tol"]["primal"]
    # the GPU and the CPU oracle solved the same instances: residuals of the same magnitude
    assert r["final_residual"]["primal_mean"] > 0
    # config-5 training record: one timed TBPTT window, cell-backward roofline
    tr = r["train"]
    assert tr["value"] > 0 and tr["loss"] == tr["loss"] and tr["batch_per_gpu"] == 8
    assert tr["roofline"]["launches"] == 3 and tr["roofline"]["bound"] == "mfma"


def test_bench_two_ranks_shared_gpu():
    r = _run(["bench.py", "--batch", "4", "--steps", "1", "--warmup", "0", "--cpu-sample", "2"] + SMALL, nproc=2)
    assert r["n_gpus"] == 2 and r["config"]["global_batch"] == 8 and r["scaling"] == "weak"
    assert "cpu_baseline" not in r  # an N = 1 figure only
    assert r["value"] > 0


def test_bench_train_two_ranks_shared_gpu():
    r = _run(["bench_train.py", "--batch", "2", "--micro_batch", "1", "--steps", "1", "--warmup", "0",
              "--num_var", "32", "--num_ineq", "16", "--num_eq", "16", "--hidden_dim", "32", "--outer_T", "2"],
             nproc=2)
    assert r["n_gpus"] == 2 and r["value"] > 0 and r["loss"] == r["loss"]


def test_bench_gpus_flag_starts_the_ranks():
    """The driver's command form: plain `python bench.py --gpus 2` (no launcher) must run two ranks
    (here sharing cuda:0 over gloo) and report n_gpus 2 over the doubled global batch."""
    env = dict(os.environ, IADMM_SHARED_GPU="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--batch", "4", "--steps", "1", "--warmup", "0",
                          "--cpu-sample", "0", "--stage2-iters", "0", "--alt-f16x3", "0"] + SMALL,
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["global_batch"] == 8 and r["dist_backend"] == "gloo"


def test_bench_train_gpus_flag_starts_the_ranks():
    env = dict(os.environ, IADMM_SHARED_GPU="1")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, "bench_train.py", "--gpus", "2", "--batch", "2", "--micro_batch", "1",
                          "--steps", "1", "--warmup", "0", "--num_var", "32", "--num_ineq", "16", "--num_eq", "16",
                          "--hidden_dim", "32", "--outer_T", "2"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert r["n_gpus"] == 2 and r["dist_backend"] == "gloo" and r["allreduce_calls"] >= 1


def _need_two_gpus():
    if torch.cuda.device_count() < 2:
        pytest.skip("the RCCL path needs >= 2 GPUs (one rank per GPU)")


def test_bench_two_ranks_rccl():
    """Config 3's code path as it runs on a multi-GPU node: one rank per GPU, backend nccl (=
    RCCL), no IADMM_SHARED_GPU.  Sharded instances, barrier, max-over-ranks timing."""
    _need_two_gpus()
    r = _run(["bench.py", "--batch", "4", "--steps", "1", "--warmup", "0", "--cpu-sample", "0"] + SMALL, nproc=2,
             shared=False)
    assert r["n_gpus"] == 2 and r["config"]["global_batch"] == 8 and r["value"] > 0


def test_bench_gpus_flag_rccl():
    """`python bench.py --gpus 2` on a multi-GPU node: one rank per GPU over RCCL."""
    _need_two_gpus()
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("IADMM_SHARED_GPU", None)
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--batch", "4", "--steps", "1", "--warmup", "0",
                          "--cpu-sample", "0", "--stage2-iters", "0", "--alt-f16x3", "0"] + SMALL,
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert r["n_gpus"] == 2 and r["config"]["global_batch"] == 8 and r["dist_backend"] == "nccl"


def test_bench_train_two_ranks_rccl():
    """Config 5's code path: the gradient all-reduce over RCCL, one rank per GPU."""
    _need_two_gpus()
    r = _run(["bench_train.py", "--batch", "2", "--micro_batch", "1", "--steps", "1", "--warmup", "0",
              "--num_var", "32", "--num_ineq", "16", "--num_eq", "16", "--hidden_dim", "32", "--outer_T", "2"],
             nproc=2, shared=False)
    assert r["n_gpus"] == 2 and r["value"] > 0 and r["loss"] == r["loss"]


def test_bench_rccl_world1():
    """The RCCL branch of parallel.init on hardware with the one GPU a builder box has: a world-1
    process group over nccl (IADMM_FORCE_DIST=1), barriers through RCCL."""
    r = _run(["bench.py", "--batch", "4", "--steps", "1", "--warmup", "0", "--cpu-sample", "0"] + SMALL, nproc=1,
             shared=False, extra_env={"IADMM_FORCE_DIST": "1"}, launcher=True)
    assert r["n_gpus"] == 1 and r["value"] > 0 and r["dist_backend"] == "nccl"


def test_bench_train_rccl_world1():
    """Config 5's bucketed gradient all-reduce through RCCL (world 1: the collective runs, the
    values are unchanged)."""
    r = _run(["bench_train.py", "--batch", "2", "--micro_batch", "1", "--steps", "1", "--warmup", "0",
              "--num_var", "32", "--num_ineq", "16", "--num_eq", "16", "--hidden_dim", "32", "--outer_T", "2"],
             nproc=1, shared=False, extra_env={"IADMM_FORCE_DIST": "1"}, launcher=True)
    assert r["n_gpus"] == 1 and r["value"] > 0 and r["loss"] == r["loss"] and r["dist_backend"] == "nccl"
    assert r["allreduce_calls"] >= 1
