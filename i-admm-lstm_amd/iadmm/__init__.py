"""iadmm — MI355X-native I-ADMM-LSTM solve loop (PyTorch-ROCm host + hand-written gfx950 HIP).

Layers: ``_abi`` (ctypes binding of libiadmm.so, the C-ABI in include/iadmm.h) -> ``ops``
(tensor-level kernel wrappers) -> ``solver`` (the fused test-mode solve loop) and
``kktop`` (the lazy KKT operator returned as ``A_tild``).  The reference-compatible module
surface (models/lstm.py, models/lu.py, methods/scaling.py, utils.py, main.py) lives at the repo
root and is built on these.
"""
from . import _abi, ops  # noqa: F401

__all__ = ["_abi", "ops"]
