"""Puts the ``i-admm-lstm_amd`` package directory on sys.path so ``import iadmm`` works from the
reference-compatible modules at the repo root (the directory name is not a Python identifier)."""
import os
import sys

PKG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "i-admm-lstm_amd")
if PKG_DIR not in sys.path:
    sys.path.insert(0, PKG_DIR)
