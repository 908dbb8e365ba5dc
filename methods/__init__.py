"""Reference-compatible preconditioner module (methods/scaling.py) backed by libiadmm.so."""
import iadmm_path  # noqa: F401
