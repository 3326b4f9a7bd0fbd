"""Lowering of linear-operator trees to device-tensor pipelines.

The reference evaluates a metric such as the geoVI Newton metric

    M = (1 + J_A^T L_A^T L_B J_B)^T (1 + J_A^T L_A^T L_B J_B)

(src/minimization/kl_energies.py:147-155: GaussianEnergy(m) @ transformation
with transformation = 1 + fl.jac^T f_lh) operator by operator on Fields.
Here a tree built from the operators of the sampling hot path is lowered ONCE
per expansion point into a composition of native calls on raw device tensors:

  * latent MultiFields are packed flat buffers (packing.PackedLayout),
  * grid / data fields are plain tensors,
  * the correlated-field Jacobian (CFJacobian) runs its fused transforms,
  * runs of pointwise factors around a LOSResponse are folded into the LOS
    kernels' column / row scales (nft_los_*),
  * a sum "alpha * 1 + X" whose X ends in a CF Jacobian adjoint is folded
    into that adjoint's epilogue (out = alpha * x + X x).

Every lowered callable has the signature  f(x, acc=None, alpha=0.) -> y  with
y = op(x) + alpha * acc.  The result is the same linear map as the operator
tree; only the number of passes over HBM and of host round trips changes.
Unsupported operators make ``lower`` return None (the caller then keeps the
generic path).  FusedCG captures lowered metrics in a HIP graph."""
import torch

from . import _native
from .domain_tuple import DomainTuple
from .multi_domain import MultiDomain


def _is_real_scale(op):
    from .operators.scaling_operator import ScalingOperator
    return isinstance(op, ScalingOperator) and complex(op._factor).imag == 0


def _pointwise(op):
    """('scale', float) | ('diag', tensor) | ('id', None) for a pointwise real
    factor on a single DomainTuple, else None."""
    from .operators.diagonal_operator import DiagonalOperator
    from .operators.simple_linear_operators import GeometryRemover
    if _is_real_scale(op) and not isinstance(op.domain, MultiDomain):
        return "scale", complex(op._factor).real
    if isinstance(op, DiagonalOperator) and not op._complex:
        return "diag", op.diagonal_tensor
    if isinstance(op, GeometryRemover):
        return "id", None
    return None


def _finish(y, acc, alpha):
    if acc is None or alpha == 0.0:
        return y
    return y.add_(acc.reshape(y.shape), alpha=alpha)


class _Unsupported(Exception):
    pass


def _adj_parts(op, adjoint):
    """unwrap OperatorAdapter(adjoint) layers"""
    from .operators.operator_adapter import OperatorAdapter
    while isinstance(op, OperatorAdapter):
        if op.trafo != op.ADJOINT_BIT:
            raise _Unsupported(op)
        adjoint = not adjoint
        op = op.wrapped
    return op, adjoint


def _lower_leaf(op, adjoint):
    from .library.correlated_fields_simple import CFJacobian
    from .library.los_response import LOSResponse
    op, adjoint = _adj_parts(op, adjoint)
    if _is_real_scale(op) and isinstance(op.domain, MultiDomain):
        v = complex(op._factor).real  # packed latent buffers: padding stays zero
        if v == 1.0:
            return lambda x, acc=None, alpha=0.: _finish(x.clone(), acc, alpha)
        return lambda x, acc=None, alpha=0.: _finish(x * v, acc, alpha)
    pw = _pointwise(op)
    if pw is not None:
        kind, v = pw
        shp = (op.domain if adjoint else op.target).shape
        if kind == "id":
            return lambda x, acc=None, alpha=0.: _finish(x.reshape(shp).clone(), acc, alpha)
        if kind == "scale":
            return lambda x, acc=None, alpha=0.: _finish(x.reshape(shp) * v, acc, alpha)
        return lambda x, acc=None, alpha=0.: _finish(x.reshape(shp) * v, acc, alpha)
    if isinstance(op, CFJacobian):
        lay = op.layout
        if not adjoint:
            def f(x, acc=None, alpha=0.):
                return _finish(op._times_t(lay.views(x)), acc, alpha)
        else:
            def f(x, acc=None, alpha=0.):
                out = lay.empty()
                if acc is not None and alpha != 0.0:
                    op._adjoint_t(x, lay.views(out), lay.views(acc), alpha)
                else:
                    op._adjoint_t(x, lay.views(out))
                return out
        return f
    if isinstance(op, LOSResponse):
        return _los(op, adjoint, None, None, 1.0)
    raise _Unsupported(op)


def _los(R, adjoint, cin, cout, scale):
    """R (or R^T) with pointwise input factor cin and output factor cout
    folded into the kernels (tensors or None) and a scalar `scale`."""
    plan = R._box_plan()
    nlos = R.target.shape[0]
    gshape = R.domain.shape
    cin = None if cin is None else cin.reshape(-1).contiguous()
    cout = None if cout is None else cout.reshape(-1).contiguous()
    if not adjoint:
        def f(x, acc=None, alpha=0.):
            y = torch.empty(nlos, dtype=x.dtype, device=x.device)
            _native.los_forward(plan, x.reshape(-1).contiguous(), y, colscale=cin, rowscale=cout, scale=scale)
            return _finish(y, acc, alpha)
    else:
        def f(x, acc=None, alpha=0.):
            out = torch.empty(gshape, dtype=x.dtype, device=x.device)
            _native.los_adjoint(plan, x.reshape(-1).contiguous(), out.view(-1), colscale=cin, rowscale=cout,
                                scale=scale)
            return _finish(out, acc, alpha)
    return f


def _fold(items):
    """product of pointwise items -> (tensor or None, float scale)"""
    t, s = None, 1.0
    for kind, v in items:
        if kind == "scale":
            s *= v
        elif kind == "diag":
            t = v if t is None else t * v
    return t, s


def _lower_chain(ops, adjoint):
    """ops: chain factors outermost first.  Returns a callable."""
    from .library.los_response import LOSResponse
    seq = [(_adj_parts(op, adjoint)) for op in (reversed(ops) if adjoint else ops)]
    # application order: innermost first
    seq = list(reversed(seq))
    fns = []
    i = 0
    while i < len(seq):
        op, adj = seq[i]
        if isinstance(op, LOSResponse):
            # absorb the pointwise run before (input side) and after (output side)
            pre = []
            while fns and fns[-1][0] == "pw":
                pre.insert(0, fns.pop()[1])
            post = []
            j = i + 1
            while j < len(seq) and _pointwise(seq[j][0]) is not None:
                post.append(_pointwise(seq[j][0]))
                j += 1
            cin, s_in = _fold(pre)
            cout, s_out = _fold(post)
            fns.append(("fn", _los(op, adj, cin, cout, s_in * s_out)))
            i = j
            continue
        pw = _pointwise(op)
        if pw is not None:
            fns.append(("pw", pw, op, adj))
            i += 1
            continue
        fns.append(("fn", _lower_any(op, adj)))
        i += 1
    # remaining pointwise runs become plain elementwise callables
    out = []
    k = 0
    while k < len(fns):
        if fns[k][0] == "pw":
            run = []
            while k < len(fns) and fns[k][0] == "pw":
                run.append(fns[k])
                k += 1
            t, s = _fold([r[1] for r in run])
            shp = (run[-1][2].domain if run[-1][3] else run[-1][2].target).shape

            def g(x, acc=None, alpha=0., t=t, s=s, shp=shp):
                y = x.reshape(shp)
                y = y * t if t is not None else y.clone()
                if s != 1.0:
                    y.mul_(s)
                return _finish(y, acc, alpha)
            out.append(g)
        else:
            out.append(fns[k][1])
            k += 1
    if not out:
        raise _Unsupported("empty chain")

    def f(x, acc=None, alpha=0.):
        y = x
        for h in out[:-1]:
            y = h(y)
        return out[-1](y, acc, alpha)
    return f


def _lower_sum(op, adjoint):
    scal = 0.0
    rest = []
    for o, neg in zip(op._ops, op._neg):
        if _is_real_scale(o):
            scal += (-1 if neg else 1) * complex(o._factor).real
        else:
            rest.append((_lower_any(o, adjoint), neg))
    if not rest:
        raise _Unsupported(op)

    def f(x, acc=None, alpha=0.):
        f0, n0 = rest[0]
        if n0:
            y = f0(x)
            y.neg_()
            if scal != 0.0:
                y.add_(x.reshape(y.shape), alpha=scal)
        else:
            y = f0(x, x if scal != 0.0 else None, scal)
        for fi, ng in rest[1:]:
            y.add_(fi(x).reshape(y.shape), alpha=-1.0 if ng else 1.0)
        return _finish(y, acc, alpha)
    return f


def _lower_any(op, adjoint=False):
    from .operators.chain_operator import ChainOperator
    from .operators.sandwich_operator import SandwichOperator
    from .operators.sum_operator import SumOperator
    op, adjoint = _adj_parts(op, adjoint)
    if isinstance(op, SandwichOperator):
        bun, cheese = op._bun, op._cheese
        fb = _lower_any(bun, False)
        fc = _lower_any(cheese, False)
        fbt = _lower_any(bun, True)

        def f(x, acc=None, alpha=0.):
            return fbt(fc(fb(x)), acc, alpha)
        return f
    if isinstance(op, ChainOperator):
        return _lower_chain(list(op._ops), adjoint)
    if isinstance(op, SumOperator):
        return _lower_sum(op, adjoint)
    return _lower_leaf(op, adjoint)


def lower(op, adjoint=False):
    """Lowered callable for `op` (see module docstring) or None."""
    try:
        return _lower_any(op, adjoint)
    except _Unsupported:
        return None


class LoweredMetric:
    """metric_flat interface of FusedCG for a lowered endomorphic operator on
    a latent MultiDomain: q = shift * d + A d on packed buffers."""

    def __init__(self, A, fn, layout):
        self.A = A
        self.fn = fn
        self.layout = layout
        self.device = layout.device
        self.domain = A.domain

    def metric_flat(self, d, q, W, shift):
        y = self.fn(d, d if shift != 0.0 else None, shift)
        q.copy_(y.reshape(-1)[:q.numel()] if y.numel() >= q.numel() else y)

    def metric_flat_batch(self, D, Q, W, shift):
        """rows one after another (the batched CG loop with one right-hand
        side runs exactly metric_flat)"""
        for j in range(D.shape[0]):
            self.metric_flat(D[j], Q[j], W, shift)
        return Q


def lowered_metric(A):
    """LoweredMetric for A if A is an endomorphic operator on a latent
    MultiDomain whose whole tree lowers, else None."""
    from .library.correlated_fields_simple import CFJacobian
    if not isinstance(A.domain, MultiDomain) or A.domain != A.target:
        return None
    fn = lower(A)
    if fn is None:
        return None
    # the packed layout of the CF Jacobian that owns this latent domain
    lay = _find_layout(A)
    if lay is None or list(lay.keys) != list(A.domain.keys()):
        return None
    del CFJacobian
    return LoweredMetric(A, fn, lay)


def _find_layout(op):
    from .library.correlated_fields_simple import CFJacobian
    from .operators.chain_operator import ChainOperator
    from .operators.operator_adapter import OperatorAdapter
    from .operators.sandwich_operator import SandwichOperator
    from .operators.sum_operator import SumOperator
    stack = [op]
    while stack:
        o = stack.pop()
        if isinstance(o, CFJacobian):
            return o.layout
        if isinstance(o, OperatorAdapter):
            stack.append(o.wrapped)
        elif isinstance(o, SandwichOperator):
            stack += [o._bun, o._cheese]
        elif isinstance(o, (ChainOperator, SumOperator)):
            stack += list(o._ops)
    return None


__all__ = ["lower", "lowered_metric", "LoweredMetric", "DomainTuple"]
