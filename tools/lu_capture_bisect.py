"""VERDICT r05 item 8, second probe: tools/capture_probe.hip's eight stream patterns all capture and
replay, so the crash needs something of the real factorization.  One capture per process of the
guard-free variant (IADMM_LIB_PATH=tools/var_lu_capture.so), argv: mode N B flags
  mode torch: torch.cuda.graph around ops.lu_factor (as tests/test_abi_concurrency_gpu.py does)
  mode raw:   hipStreamBeginCapture / EndCapture / GraphInstantiate through ctypes, no torch graph
flags 4 = IADMM_LU_RANK128 (the look-ahead's fork / join at any N).  Prints the node count."""
import ctypes
import faulthandler
import json
import os
import sys

faulthandler.enable()
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "i-admm-lstm_amd"))
import torch  # noqa: E402
from iadmm import ops  # noqa: E402

mode, N, B, flags = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
g = torch.Generator(device="cuda").manual_seed(N)
K = torch.randn(B, N, N, generator=g, device="cuda")
K[:, 0, 0] = 0.0
ref, rpiv, _ = ops.lu_factor(K.clone(), flags=flags)
torch.cuda.synchronize()
s = torch.cuda.Stream()
ws = ops.lu_factor_ws(B, N, K.device)
A = K.clone()
with torch.cuda.stream(s):
    ops.lu_factor(A.clone(), ws=ws, flags=flags)  # warm-up: this stream's context
s.synchronize()
hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch loaded (same soname), not a second one
out = dict(mode=mode, N=N, B=B, flags=flags)
print("[bisect]", out, "capturing", flush=True)
if mode == "torch":
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        LU, piv, info = ops.lu_factor(A, ws=ws, flags=flags)
    print("[bisect] captured", flush=True)
    gr.replay()
else:
    st = ctypes.c_void_p(s.cuda_stream)
    assert hip.hipStreamBeginCapture(st, 0) == 0  # hipStreamCaptureModeGlobal
    with torch.cuda.stream(s):
        LU, piv, info = ops.lu_factor(A, ws=ws, flags=flags)
    graph = ctypes.c_void_p()
    print("[bisect] end capture", flush=True)
    rc = hip.hipStreamEndCapture(st, ctypes.byref(graph))
    nn = ctypes.c_size_t()
    hip.hipGraphGetNodes(graph, None, ctypes.byref(nn))
    out.update(end_rc=rc, nodes=nn.value)
    print("[bisect] end rc", rc, "nodes", nn.value, "instantiate", flush=True)
    ex = ctypes.c_void_p()
    out["inst_rc"] = hip.hipGraphInstantiate(ctypes.byref(ex), graph, None, None, ctypes.c_size_t(0))
    print("[bisect] instantiated", out["inst_rc"], flush=True)
    out["launch_rc"] = hip.hipGraphLaunch(ex, st)
s.synchronize()
out["bitwise"] = bool(torch.equal(LU, ref) and torch.equal(piv, rpiv))
print(json.dumps(out), flush=True)
