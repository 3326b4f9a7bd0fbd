"""Global configuration (mirror of src/config.py:3-40) plus the compute device.

``hartley_convention``: "non_canonical_hartley" (default, Re F + Im F) or
"canonical_hartley" (Re F - Im F); aliases "ducc_hartley" / "ducc_fht".
"""
import os

import torch

_config = dict(hartley_convention="non_canonical_hartley")
_device = None
# storage precision of the fused CG loops (build extension, BASELINE config
# C5): "fp64" (default, the reference's arithmetic) or "fp32" (vectors and
# grid operands in fp32, every reduction and all CG scalars in fp64)
_cg_precision = "fp64"


def update(key, value, /):
    global _config
    if not isinstance(key, str):
        raise TypeError(f"key must be a string; got {key!r}")
    key = key.lower()
    if key == "hartley_convention":
        if not isinstance(value, str):
            raise TypeError(f"value to {key!r} must be a string; got {value!r}")
        if value in ("ducc_hartley", "non_canonical_hartley"):
            value = "non_canonical_hartley"
        elif value in ("ducc_fht", "canonical_hartley"):
            value = "canonical_hartley"
        else:
            raise ValueError(f"invalid value to {key!r}; got {value!r}")
    else:
        raise ValueError(f"invalid key; got {key!r}")
    _config[key] = value


def set_cg_precision(p):
    global _cg_precision
    if p not in ("fp64", "fp32"):
        raise ValueError(f"cg precision must be 'fp64' or 'fp32'; got {p!r}")
    _cg_precision = p


def cg_dtype():
    return torch.float32 if _cg_precision == "fp32" else torch.float64


def hartley_convention_code():
    return 0 if _config["hartley_convention"] == "non_canonical_hartley" else 1


def device():
    """Device on which Fields are created: this process's GPU (LOCAL_RANK) if
    one is visible, else the CPU (host logic only: hot-path ops raise there)."""
    global _device
    if _device is None:
        if torch.cuda.is_available():
            _device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
        else:
            _device = torch.device("cpu")
    return _device


def set_device(dev):
    global _device
    _device = torch.device(dev)
