"""One process per GPU from a plain ``python bench.py --gpus N`` command line.

``bench.py`` / ``bench_train.py`` are launched either by ``torch.distributed.run`` (WORLD_SIZE set:
each process is one rank) or directly.  Run directly with ``--gpus N > 1``, the script must not
measure one rank and call it N: :func:`relaunch` starts ``python -m torch.distributed.run
--nproc-per-node N <script> <same args>`` as a CHILD process (never ``exec``: the parent has not
touched the GPU, but a child keeps the rule simple and the exit status explicit), lets the child's
rank 0 write its JSON line to the inherited stdout and exits with the child's status.

This module imports nothing but the standard library and is loaded before ``torch.cuda`` or the
``iadmm`` package is touched, so the parent process never initialises HIP.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys


class LaunchError(SystemExit):
    """A --gpus / WORLD_SIZE mismatch: exits non-zero with the message."""


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def child_command(script, argv, gpus, port=None):
    """The torch.distributed.run command line of the N-rank child (rendezvous on 127.0.0.1)."""
    port = free_port() if port is None else port
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(gpus)}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), script] + list(argv)


def check_world(gpus, env=None):
    """Under a launcher (WORLD_SIZE set) the world must equal --gpus; returns the world size or
    None when no launcher started this process."""
    env = os.environ if env is None else env
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return None
    if int(ws) != int(gpus):
        raise LaunchError(f"--gpus {gpus} but WORLD_SIZE={ws}: the launcher started a different number of "
                          f"ranks than the command asks for (pass --gpus {ws}, or launch {gpus} ranks)")
    return int(ws)


def relaunch(script, argv, gpus):
    """Return normally when this process should run the benchmark itself (under a launcher, or
    --gpus 1).  Otherwise run the N-rank child and exit with its return code."""
    if check_world(gpus) is not None or int(gpus) <= 1:
        return
    cmd = child_command(script, argv, gpus)
    print(f"[launch] starting {gpus} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    child = subprocess.Popen(cmd, env=dict(os.environ))

    sent = []

    def forward(signum, _frame):  # a `kill <pid>` SIGTERM reaches the ranks through the launcher, once
        if sent:
            return
        sent.append(signum)
        try:
            child.send_signal(signum)
        except ProcessLookupError:
            pass

    signal.signal(signal.SIGTERM, forward)
    # Ctrl-C reaches the child directly (same process group); forwarding it as well would give
    # torch.distributed.run a second SIGINT in the middle of its worker cleanup
    signal.signal(signal.SIGINT, signal.SIG_IGN)
    rc = child.wait()
    sys.exit(rc if rc >= 0 else 128 - rc)
