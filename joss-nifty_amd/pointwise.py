"""Pointwise functions and their derivatives on torch tensors
(mirror of src/pointwise.py:130-155; note NIFTy's ``sigmoid`` is
0.5 + 0.5 tanh(x), not the logistic function)."""
import math

import torch


def _sqrt(v):
    t = torch.sqrt(v)
    return t, 0.5 / t


def _sinc(v):
    t = torch.sinc(v)
    pv = math.pi * v
    d = torch.where(v == 0, torch.zeros_like(v), (torch.cos(pv) - t) / torch.where(v == 0, torch.ones_like(v), v))
    return t, d


def _expm1(v):
    t = torch.expm1(v)
    return t, t + 1.


def _tanh(v):
    t = torch.tanh(v)
    return t, 1. - t * t


def _sigmoid(v):
    t = torch.tanh(v)
    return 0.5 + 0.5 * t, 0.5 * (1. - t * t)


def _reciprocal(v):
    t = 1. / v
    return t, -t * t


def _abs(v):
    return torch.abs(v), torch.sign(v)


def _sign(v):
    return torch.sign(v), torch.zeros_like(v)


def _power(v, p):
    t = torch.pow(v, p)
    return t, p * torch.pow(v, p - 1)


def _clip(v, a_min=None, a_max=None):
    t = torch.clip(v, a_min, a_max)
    d = torch.ones_like(v)
    if a_min is not None:
        d = torch.where(v < a_min, torch.zeros_like(v), d)
    if a_max is not None:
        d = torch.where(v > a_max, torch.zeros_like(v), d)
    return t, d


def softplus(v):
    return torch.log(1. + torch.exp(v))


def _softplus(v):
    t = torch.exp(v)
    return torch.log(1. + t), t / (1. + t)


def exponentiate(v, base):
    return torch.pow(base, v)


def _exponentiate(v, base):
    t = torch.pow(base, v)
    return t, math.log(base) * t


def _step(v, grad):
    if grad:
        return torch.where(v > 0, 1., 0.).to(v.dtype), torch.zeros_like(v)
    return torch.where(v > 0, 1., 0.).to(v.dtype)


ptw_dict = {
    "sqrt": (torch.sqrt, _sqrt),
    "sin": (torch.sin, lambda v: (torch.sin(v), torch.cos(v))),
    "cos": (torch.cos, lambda v: (torch.cos(v), -torch.sin(v))),
    "tan": (torch.tan, lambda v: (torch.tan(v), 1. / torch.cos(v) ** 2)),
    "sinc": (torch.sinc, _sinc),
    "exp": (torch.exp, lambda v: (lambda t: (t, t))(torch.exp(v))),
    "expm1": (torch.expm1, _expm1),
    "log": (torch.log, lambda v: (torch.log(v), 1. / v)),
    "log10": (torch.log10, lambda v: (torch.log10(v), (1. / math.log(10.)) / v)),
    "log1p": (torch.log1p, lambda v: (torch.log1p(v), 1. / (1. + v))),
    "sinh": (torch.sinh, lambda v: (torch.sinh(v), torch.cosh(v))),
    "cosh": (torch.cosh, lambda v: (torch.cosh(v), torch.sinh(v))),
    "tanh": (torch.tanh, _tanh),
    "sigmoid": (lambda v: 0.5 + 0.5 * torch.tanh(v), _sigmoid),
    "reciprocal": (lambda v: 1. / v, _reciprocal),
    "abs": (torch.abs, _abs),
    "absolute": (torch.abs, _abs),
    "sign": (torch.sign, _sign),
    "power": (torch.pow, _power),
    "clip": (torch.clip, _clip),
    "softplus": (softplus, _softplus),
    "exponentiate": (exponentiate, _exponentiate),
    "arctan": (torch.arctan, lambda v: (torch.arctan(v), 1. / (1. + v ** 2))),
    "unitstep": (lambda v: _step(v, False), lambda v: _step(v, True)),
}
