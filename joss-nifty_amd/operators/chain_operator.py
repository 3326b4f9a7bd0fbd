"""ChainOperator: product of linear operators with the reference's
simplifications (scalar folding into diagonals, diagonal merging;
src/operators/chain_operator.py:24-149)."""
from .. import utilities
from .linear_operator import LinearOperator


class ChainOperator(LinearOperator):
    def __init__(self, ops, _callingfrommake=False):
        if not _callingfrommake:
            raise NotImplementedError
        self._ops = ops
        self._capability = self._all_ops
        for op in ops:
            self._capability &= op.capability
        self._domain = self._ops[-1].domain
        self._target = self._ops[0].target

    @staticmethod
    def simplify(ops):
        from .diagonal_operator import DiagonalOperator
        from .scaling_operator import ScalingOperator
        from .simple_linear_operators import NullOperator
        from .block_diagonal_operator import BlockDiagonalOperator
        for i in range(len(ops) - 1):
            utilities.check_object_identity(ops[i + 1].target, ops[i].domain)
        opsnew = []
        for op in ops:
            opsnew += op._ops if isinstance(op, ChainOperator) else [op]
        ops = opsnew
        if any(isinstance(op, NullOperator) for op in ops):
            ops = (NullOperator(ops[-1].domain, ops[0].target),)
        fct = 1.
        opsnew = []
        lastdom = ops[-1].domain
        for op in ops:
            if isinstance(op, ScalingOperator) and complex(op._factor).imag == 0:
                fct *= complex(op._factor).real
            else:
                opsnew.append(op)
        if fct != 1.:
            for i in range(len(opsnew)):
                if isinstance(opsnew[i], DiagonalOperator):
                    opsnew[i] = opsnew[i]._scale(fct)
                    fct = 1.
                    break
        if fct != 1 or len(opsnew) == 0:
            opsnew.append(ScalingOperator(lastdom, fct))
        ops = opsnew
        opsnew = []
        for op in ops:
            if len(opsnew) > 0 and isinstance(opsnew[-1], DiagonalOperator) and isinstance(op, DiagonalOperator):
                opsnew[-1] = opsnew[-1]._combine_prod(op)
            else:
                opsnew.append(op)
        ops = opsnew
        opsnew = []
        for op in ops:
            if (len(opsnew) > 0 and isinstance(opsnew[-1], BlockDiagonalOperator)
                    and isinstance(op, BlockDiagonalOperator)):
                opsnew[-1] = opsnew[-1]._combine_chain(op)
            else:
                opsnew.append(op)
        return opsnew

    @staticmethod
    def make(ops):
        ops = tuple(ops)
        if len(ops) == 0:
            raise ValueError("ops is empty")
        ops = ChainOperator.simplify(ops)
        if len(ops) == 1:
            return ops[0]
        return ChainOperator(ops, _callingfrommake=True)

    def _flip_modes(self, trafo):
        ADJ, INV = self.ADJOINT_BIT, self.INVERSE_BIT
        if trafo == 0:
            return self
        if trafo == ADJ or trafo == INV:
            return self.make([op._flip_modes(trafo) for op in reversed(self._ops)])
        if trafo == ADJ | INV:
            return self.make([op._flip_modes(trafo) for op in self._ops])
        raise ValueError("invalid operator transformation")

    def apply(self, x, mode):
        self._check_mode(mode)
        t_ops = self._ops if mode & self._backwards else reversed(self._ops)
        for op in t_ops:
            x = op.apply(x, mode)
        return x

    @property
    def ops(self):
        return self._ops

    def __repr__(self):
        return "ChainOperator:\n" + utilities.indent("\n".join(repr(op) for op in self._ops))
