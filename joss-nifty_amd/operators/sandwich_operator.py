"""SandwichOperator: bun^dagger cheese bun (src/operators/sandwich_operator.py).

MI355X fusion hook: when the bun is a chain  D_k ... D_1 J  whose rightmost
factor J is a fused model Jacobian (e.g. the correlated-field Jacobian,
library/correlated_fields_simple.py) and every other factor is pointwise on
J's target grid (diagonal, scaling, geometry removal), the whole sandwich
J^T W J with W = cheese * prod D_i^2 is evaluated by J's fused native
pipeline (J.sandwich_apply) instead of operator by operator.  Results are the
same linear map; only the number of HBM passes changes."""
import torch

from .. import utilities
from .chain_operator import ChainOperator
from .diagonal_operator import DiagonalOperator
from .endomorphic_operator import EndomorphicOperator
from .linear_operator import LinearOperator
from .scaling_operator import ScalingOperator


def _pointwise_weight(ops, cheese):
    """Return W (device tensor broadcastable to the grid) if `ops` (bun factors
    applied after J, outermost first) and `cheese` are all pointwise, else None."""
    from .simple_linear_operators import GeometryRemover
    w = None
    for op in ops:
        if isinstance(op, ScalingOperator):
            f = complex(op._factor)
            if f.imag != 0:
                return None
            w = (f.real ** 2) if w is None else w * f.real ** 2
        elif isinstance(op, DiagonalOperator):
            if op._complex:
                return None
            d = op.diagonal_tensor
            w = d * d if w is None else w * d * d
        elif isinstance(op, GeometryRemover):
            continue
        else:
            return None
    if isinstance(cheese, ScalingOperator):
        f = complex(cheese._factor)
        if f.imag != 0:
            return None
        w = f.real if w is None else w * f.real
    elif isinstance(cheese, DiagonalOperator):
        if cheese._complex:
            return None
        w = cheese.diagonal_tensor if w is None else w * cheese.diagonal_tensor
    else:
        return None
    return w


def _pointwise_diag(ops):
    """Product of the (real) diagonals of `ops` (tensor, float or None = 1),
    or False if any factor is not pointwise."""
    from .simple_linear_operators import GeometryRemover
    d = None
    for op in ops:
        if isinstance(op, ScalingOperator):
            f = complex(op._factor)
            if f.imag != 0:
                return False
            d = f.real if d is None else d * f.real
        elif isinstance(op, DiagonalOperator):
            if op._complex:
                return False
            t = op.diagonal_tensor
            d = t if d is None else d * t
        elif isinstance(op, GeometryRemover):
            continue
        else:
            return False
    return d


def _fused_response_middle(left, cheese, fct):
    """Middle M^T C M for left = [data-side pointwise..., R, grid-side
    pointwise...] with R providing `fused_middle` (LOSResponse), else None."""
    ir = [i for i, op in enumerate(left) if hasattr(op, "fused_middle")]
    if len(ir) != 1:
        return None
    i = ir[0]
    c = _pointwise_weight(left[:i], cheese)
    dr = _pointwise_diag(left[i + 1:])
    if c is None or dr is False:
        return None
    if dr is not None and not torch.is_tensor(dr):
        fct *= float(dr) ** 2
        dr = None
    R = left[i]
    if dr is not None and dr.numel() != R.domain.size:
        return None
    if torch.is_tensor(c) and c.numel() not in (1, R.target.size):
        return None
    return R.fused_middle(dr, c, fct)


class SandwichOperator(EndomorphicOperator):
    def __init__(self, bun, cheese, op, _callingfrommake=False):
        if not _callingfrommake:
            raise NotImplementedError
        self._bun = bun
        self._cheese = cheese
        self._op = op
        self._domain = op.domain
        self._capability = op._capability
        self._fused = None
        self._detect_fusion()

    def _detect_fusion(self):
        bun = self._bun
        ops = list(bun._ops) if isinstance(bun, ChainOperator) else [bun]
        cores = [i for i, op in enumerate(ops) if hasattr(op, "sandwich_apply")]
        if len(cores) != 1:
            return
        core = ops[cores[0]]
        # factors applied before the core (right of it) may only be scalars
        # (ChainOperator.simplify moves folded scalars to the end of the chain)
        right = ops[cores[0] + 1:]
        if not all(isinstance(op, ScalingOperator) for op in right):
            return
        w = _pointwise_weight(ops[:cores[0]] + right, self._cheese)
        if w is None:
            # non-pointwise middle (e.g. a line-of-sight response): the model
            # Jacobian halves stay fused, the middle M^T C M runs through the
            # generic operator tree on J's target
            if not all(isinstance(op, ScalingOperator) and complex(op._factor).imag == 0 for op in right):
                return
            fct = 1.
            for op in right:
                fct *= complex(op._factor).real ** 2
            left = ops[:cores[0]]
            fm = _fused_response_middle(left, self._cheese, fct)
            if fm is not None:
                self._fused = (core, fm)
                return
            mid = ChainOperator.make(left) if len(left) > 0 else None
            cheese = self._cheese
            tgt = core.target

            def middle(s):
                from ..field import Field
                f = Field(tgt, s)
                if mid is None:
                    r = cheese(f)
                else:
                    r = mid.adjoint_times(cheese(mid(f)))
                return r.val * fct if fct != 1. else r.val
            self._fused = (core, middle)
            return
        if not torch.is_tensor(w):
            w = torch.full(core.target.shape, float(w), dtype=torch.float64, device=core.device)
        else:
            w = w.expand(core.target.shape).contiguous()
        self._fused = (core, w)

    @staticmethod
    def make(bun, cheese=None, sampling_dtype=None):
        if isinstance(cheese, SandwichOperator):
            old_cheese = cheese
            cheese = old_cheese._cheese
            bun = old_cheese._bun @ bun
        if not isinstance(bun, LinearOperator):
            raise TypeError("bun must be a linear operator")
        if cheese is not None and not isinstance(cheese, LinearOperator):
            raise TypeError("cheese must be a linear operator or None")
        if cheese is None:
            cheese = ScalingOperator(bun.target, 1., sampling_dtype)
        if isinstance(bun, ScalingOperator):
            fct = abs(bun._factor) ** 2
            if fct == 1.:
                return cheese
            op = cheese.scale(fct)
        else:
            op = bun.adjoint @ cheese @ bun
        return SandwichOperator(bun, cheese, op, _callingfrommake=True)

    @property
    def fused(self):
        """(fused core Jacobian, pointwise weight W) or None."""
        return self._fused

    def apply(self, x, mode):
        if self._fused is not None and mode in (self.TIMES, self.ADJOINT_TIMES):
            self._check_input(x, mode)
            core, w = self._fused
            return core.sandwich_apply(x, w)
        return self._op.apply(x, mode)

    def draw_sample(self, from_inverse=False):
        if from_inverse:
            if self._bun.capability & self._bun.INVERSE_TIMES:
                try:
                    s = self._cheese.draw_sample(from_inverse)
                    return self._bun.inverse_times(s)
                except NotImplementedError:
                    pass
            raise NotImplementedError("cannot draw from inverse of this operator")
        return self._bun.adjoint_times(self._cheese.draw_sample(from_inverse))

    def get_sqrt(self):
        if self._cheese is None:
            return self._bun
        return self._cheese.get_sqrt() @ self._bun

    def __repr__(self):
        return "SandwichOperator:\n" + utilities.indent(
            "Cheese:\n" + repr(self._cheese) + "\nBun:\n" + repr(self._bun))
