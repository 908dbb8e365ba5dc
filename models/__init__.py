"""Reference-compatible model modules (models/lstm.py, models/lu.py) backed by libiadmm.so."""
import iadmm_path  # noqa: F401
