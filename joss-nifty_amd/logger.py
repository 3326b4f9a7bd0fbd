"""Logger named like the reference's ('NIFTy8', src/logger.py)."""
import logging


def _make():
    lg = logging.getLogger("NIFTy8")
    lg.setLevel(logging.DEBUG)
    lg.propagate = False
    if not lg.handlers:
        ch = logging.StreamHandler()
        ch.setLevel(logging.WARNING)
        lg.addHandler(ch)
    return lg


logger = _make()
