"""SumOperator with the reference's scalar/diagonal folding
(src/operators/sum_operator.py:64-234)."""
from collections import defaultdict

from .. import utilities
from .linear_operator import LinearOperator


class SumOperator(LinearOperator):
    def __init__(self, ops, neg, dom, tgt, _callingfrommake=False):
        if not _callingfrommake:
            raise NotImplementedError
        self._domain = dom
        self._target = tgt
        self._ops = ops
        self._neg = neg
        self._capability = self.TIMES | self.ADJOINT_TIMES
        for op in ops:
            self._capability &= op.capability

    @staticmethod
    def simplify(ops, neg):
        from ..sugar import domain_union
        from .block_diagonal_operator import BlockDiagonalOperator
        from .diagonal_operator import DiagonalOperator
        from .scaling_operator import ScalingOperator
        opsnew, negnew = [], []
        for op, ng in zip(ops, neg):
            if isinstance(op, SumOperator):
                opsnew += op._ops
                negnew += [not n for n in op._neg] if ng else list(op._neg)
            else:
                opsnew.append(op)
                negnew.append(ng)
        ops, neg = opsnew, negnew
        srt = defaultdict(list)
        for op, ng in zip(ops, neg):
            srt[(op.domain, op.target)].append((op, ng))
        xxops, xxneg = [], []
        for opset in srt.values():
            tot = 0.
            opsnew, negnew, dtype = [], [], []
            for op, ng in opset:
                if isinstance(op, ScalingOperator):
                    tot += op._factor * (-1 if ng else 1)
                    dtype.append(op._dtype)
                else:
                    opsnew.append(op)
                    negnew.append(ng)
            lastdom = opset[0][0].domain
            if len(dtype) > 0:
                dtype = dtype[0] if all(dtype[0] == ss for ss in dtype) else None
            else:
                dtype = None
            if tot != 0.:
                for i in range(len(opsnew)):
                    if isinstance(opsnew[i], DiagonalOperator):
                        if opsnew[i]._dtype != dtype:
                            continue
                        tot *= (-1 if negnew[i] else 1)
                        opsnew[i] = opsnew[i]._add(tot)
                        tot = 0.
                        break
            if tot != 0 or len(opsnew) == 0:
                opsnew.append(ScalingOperator(lastdom, tot, dtype))
                negnew.append(False)
            ops, neg = opsnew, negnew
            processed = [False] * len(ops)
            opsnew, negnew = [], []
            for i in range(len(ops)):
                if not processed[i]:
                    if isinstance(ops[i], DiagonalOperator):
                        op, opneg = ops[i], neg[i]
                        for j in range(i + 1, len(ops)):
                            if isinstance(ops[j], DiagonalOperator) and ops[i]._dtype == ops[j]._dtype:
                                op = op._combine_sum(ops[j], opneg, neg[j])
                                opneg = False
                                processed[j] = True
                        opsnew.append(op)
                        negnew.append(opneg)
                    else:
                        opsnew.append(ops[i])
                        negnew.append(neg[i])
            ops, neg = opsnew, negnew
            processed = [False] * len(ops)
            opsnew, negnew = [], []
            for i in range(len(ops)):
                if not processed[i]:
                    if isinstance(ops[i], BlockDiagonalOperator):
                        op, opneg = ops[i], neg[i]
                        for j in range(i + 1, len(ops)):
                            if isinstance(ops[j], BlockDiagonalOperator):
                                op = op._combine_sum(ops[j], opneg, neg[j])
                                opneg = False
                                processed[j] = True
                        opsnew.append(op)
                        negnew.append(opneg)
                    else:
                        opsnew.append(ops[i])
                        negnew.append(neg[i])
            xxops += opsnew
            xxneg += negnew
        dom = domain_union([op.domain for op in xxops])
        tgt = domain_union([op.target for op in xxops])
        return xxops, xxneg, dom, tgt

    @staticmethod
    def make(ops, neg):
        ops, neg = tuple(ops), tuple(neg)
        if len(ops) == 0:
            raise ValueError("ops is empty")
        if len(ops) != len(neg):
            raise ValueError("length mismatch between ops and neg")
        ops, neg, dom, tgt = SumOperator.simplify(ops, neg)
        if len(ops) == 1:
            return -ops[0] if neg[0] else ops[0]
        return SumOperator(ops, neg, dom, tgt, _callingfrommake=True)

    @property
    def adjoint(self):
        return self.make([op.adjoint for op in self._ops], self._neg)

    def apply(self, x, mode):
        self._check_mode(mode)
        res = None
        for op, neg in zip(self._ops, self._neg):
            tmp = op.apply(x.extract(op._dom(mode)), mode)
            if res is None:
                res = -tmp if neg else tmp
            else:
                res = res.flexible_addsub(tmp, neg)
        return res

    def draw_sample(self, from_inverse=False):
        if from_inverse:
            raise NotImplementedError("cannot draw from inverse of this operator")
        res = None
        for op in self._ops:
            from ..sugar import from_random  # noqa: F401
            tmp = op.draw_sample(from_inverse)
            res = tmp if res is None else res.unite(tmp)
        return res

    def __repr__(self):
        subs = "\n".join(repr(op) for op in self._ops)
        return "SumOperator:\n" + utilities.indent(subs)
