"""Run one tools/capture_probe.hip variant inside a python process that has initialised torch, so the probe
library binds to torch's bundled HIP runtime (what libiadmm.so runs on in every python caller).
Usage: python tools/capture_probe_torch.py <probe.so> <variant>"""
import ctypes
import faulthandler
import sys

faulthandler.enable()
import torch  # noqa: E402

torch.zeros(1, device="cuda")
lib = ctypes.CDLL(sys.argv[1])
maps = open("/proc/self/maps").read()
print("hip runtimes mapped:", sorted({ln.split()[-1] for ln in maps.splitlines() if "amdhip64" in ln}), flush=True)
rc = lib.capture_probe_run(int(sys.argv[2]))
sys.stdout.flush()
sys.exit(rc)
