"""`python bench.py --gpus N` must run N ranks (iadmm/launch.py): the parent starts a
torch.distributed.run child before anything touches the GPU, a launcher/--gpus mismatch fails
loudly, and the child's rank-0 line reaches the parent's stdout.  CPU only (gloo for the relay)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

import iadmm_path  # noqa: F401
from iadmm import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("script", ["bench.py", "bench_train.py"])
def test_gpus_world_size_mismatch_exits_nonzero(script):
    env = dict(os.environ, WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, script, "--gpus", "2"], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode != 0
    assert "WORLD_SIZE=4" in out.stderr


def test_check_world():
    assert launch.check_world(3, {}) is None
    assert launch.check_world(2, {"WORLD_SIZE": "2"}) == 2
    with pytest.raises(SystemExit):
        launch.check_world(8, {"WORLD_SIZE": "1"})


def test_child_command_shape():
    cmd = launch.child_command("/x/bench.py", ["--gpus", "8", "--steps", "3"], 8, port=29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5] == "/x/bench.py"


def test_relaunch_runs_n_ranks_and_relays_rank0(tmp_path):
    """A stand-in script with bench.py's launch logic: run plainly with --gpus 2 it must come back
    as two ranks of one gloo world, rank 0 printing the single JSON line, exit status 0."""
    script = tmp_path / "probe.py"
    script.write_text(textwrap.dedent(f"""
        import argparse, json, os, sys
        sys.path.insert(0, {os.path.join(ROOT, "i-admm-lstm_amd")!r})
        from iadmm import launch
        ap = argparse.ArgumentParser(); ap.add_argument("--gpus", type=int, default=1)
        a = ap.parse_args()
        launch.relaunch(os.path.abspath(sys.argv[0]), sys.argv[1:], a.gpus)
        import torch, torch.distributed as dist
        dist.init_process_group("gloo")
        t = torch.tensor([float(dist.get_rank() + 1)])
        dist.all_reduce(t)
        if dist.get_rank() == 0:
            print(json.dumps({{"world": dist.get_world_size(), "sum": float(t)}}), flush=True)
        dist.destroy_process_group()
    """))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, str(script), "--gpus", "2"], env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    assert json.loads(lines[0]) == {"world": 2, "sum": 3.0}


def test_relaunch_propagates_failure(tmp_path):
    script = tmp_path / "fail.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys
        sys.path.insert(0, {os.path.join(ROOT, "i-admm-lstm_amd")!r})
        from iadmm import launch
        launch.relaunch(os.path.abspath(sys.argv[0]), sys.argv[1:], 2)
        sys.exit(3)
    """))
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0
