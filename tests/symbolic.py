"""Symbolic tensors for the structural pin of the hGRU oracle (test infrastructure only).

A ``Sym`` is a node of a hash-consed expression DAG.  The same vocabulary is produced from two
sides and compared by Merkle hash:

* ``tools/extract_hgru.py`` evaluates the reference's own method bodies
  (``/root/reference/hgru_module.py:9-959``, ``/root/reference/hgru_pose.py:8-216``) as an AST,
  with a TF1 stand-in that builds ``Sym`` nodes instead of graph ops;
* ``oracle/hgru_ref.py`` is run with ``Sym`` inputs (its conv / pool primitives swapped for
  symbolic ones; their numerics are pinned separately by ``tests/test_oracle.py``).

Canonical form: sums and products are flattened, their numeric constants folded, and their
operands ordered by hash (commutativity); ``a - b`` is ``a + (-1)*b``; ``a / b`` is
``a * b**-1``; ``max(x, 0)`` is ``relu(x)``.  Nothing else is rewritten, so the two sides agree
only if they apply the same ops, in the same nesting, to the same named variables and inputs.
"""
from __future__ import annotations

import hashlib
import numbers

import numpy as np

COMMUTATIVE = ("add", "mul")


class Sym:
    __array_priority__ = 1000
    __slots__ = ("op", "args", "shape", "h")

    def __init__(self, op, args, shape):
        self.op = op
        self.args = tuple(args)
        self.shape = tuple(shape) if shape is not None else None
        parts = [op]
        for a in self.args:
            parts.append(a.h if isinstance(a, Sym) else "=" + repr(a))
        if op in COMMUTATIVE:
            parts = [op] + sorted(parts[1:])
        self.h = hashlib.sha1("|".join(parts).encode()).hexdigest()

    # -- numpy-ish surface the oracle touches --------------------------------------------------
    @property
    def dtype(self):
        return np.dtype(np.float64)

    @property
    def ndim(self):
        return len(self.shape)

    def astype(self, *_a, **_k):
        return self

    def copy(self):
        return self

    def reshape(self, *shape):
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        if tuple(shape) == (-1,):
            # [1, ..., 1, k] -> [k] broadcasts identically against an NHWC tensor: not an op
            if self.shape is not None and all(d == 1 for d in self.shape[:-1]):
                return self
            return mk("flatten_all", [self], (-1,))
        if len(shape) == 2 and shape[1] == -1 and self.shape and shape[0] == self.shape[0]:
            return flatten(self)
        raise NotImplementedError(f"reshape {self.shape} -> {shape}")

    def __getitem__(self, idx):
        return mk("gather", [self, idx], ())

    def __add__(self, o):
        return add(self, o)

    __radd__ = __add__

    def __sub__(self, o):
        return add(self, neg(o))

    def __rsub__(self, o):
        return add(o, neg(self))

    def __mul__(self, o):
        return mul(self, o)

    __rmul__ = __mul__

    def __truediv__(self, o):
        return mul(self, power(o, -1))

    def __rtruediv__(self, o):
        return mul(o, power(self, -1))

    def __neg__(self):
        return neg(self)

    def __matmul__(self, o):
        return mk("matmul", [self, o], (self.shape[0], o.shape[-1]))

    def __array_ufunc__(self, ufunc, method, *inputs, **kw):
        if method != "__call__" or kw:
            return NotImplemented
        if ufunc is np.tanh:
            return tanh(inputs[0])
        if ufunc is np.exp:
            return mk("exp", [inputs[0]], inputs[0].shape)
        if ufunc is np.sqrt:
            return power(inputs[0], 0.5)
        if ufunc is np.maximum:
            return maximum(*inputs)
        if ufunc is np.minimum:
            return minimum(*inputs)
        if ufunc is np.add:
            return add(*inputs)
        if ufunc is np.subtract:
            return add(inputs[0], neg(inputs[1]))
        if ufunc is np.multiply:
            return mul(*inputs)
        if ufunc is np.true_divide:
            return mul(inputs[0], power(inputs[1], -1))
        return NotImplemented

    def __repr__(self):
        return render(self, 3)

    def __bool__(self):
        raise TypeError("a symbolic tensor has no truth value")


# ---------------------------------------------------------------------------------------------
def _num(x):
    return isinstance(x, numbers.Number) and not isinstance(x, bool) or isinstance(x, np.number)


def const(v, shape=()):
    return Sym("c", [float(v)], shape)


def lift(x):
    if isinstance(x, Sym):
        return x
    if _num(x):
        return const(x)
    if isinstance(x, np.ndarray) and x.size == 1:
        return const(float(x.reshape(-1)[0]), x.shape)
    raise TypeError(f"cannot lift {type(x)}")


def _bshape(xs):
    best = ()
    for x in xs:
        if x.shape is not None and len(x.shape) > len(best):
            best = x.shape
    return best


def mk(op, args, shape):
    return Sym(op, args, shape)


def _is_c(x, v=None):
    return isinstance(x, Sym) and x.op == "c" and (v is None or x.args[0] == v)


def add(*xs):
    xs = [lift(x) for x in xs]
    terms, c = [], 0.0
    for x in xs:
        for t in (x.args if x.op == "add" else (x,)):
            if t.op == "c":
                c += t.args[0]
            else:
                terms.append(t)
    shape = _bshape(xs)
    if c != 0.0:
        terms.append(const(c))
    if not terms:
        return const(0.0, shape)
    if len(terms) == 1:
        return terms[0]
    return Sym("add", sorted(terms, key=lambda s: s.h), shape)


def mul(*xs):
    xs = [lift(x) for x in xs]
    facs, c = [], 1.0
    for x in xs:
        for f in (x.args if x.op == "mul" else (x,)):
            if f.op == "c":
                c *= f.args[0]
            else:
                facs.append(f)
    shape = _bshape(xs)
    if c == 0.0:
        return const(0.0, shape)
    if c != 1.0:
        facs.append(const(c))
    if not facs:
        return const(c, shape)
    if len(facs) == 1:
        return facs[0]
    return Sym("mul", sorted(facs, key=lambda s: s.h), shape)


def neg(x):
    return mul(-1.0, x)


def power(x, p):
    x = lift(x)
    if x.op == "c":
        return const(x.args[0] ** p, x.shape)
    return mk("pow", [x, float(p)], x.shape)


def tanh(x):
    x = lift(x)
    return mk("tanh", [x], x.shape)


def sigmoid(x):
    x = lift(x)
    return mk("sigmoid", [x], x.shape)


def relu(x):
    x = lift(x)
    return mk("relu", [x], x.shape)


def maximum(a, b):
    a, b = lift(a), lift(b)
    if _is_c(b, 0.0):
        return relu(a)
    if _is_c(a, 0.0):
        return relu(b)
    return mk("maximum", [a, b], _bshape([a, b]))


def minimum(a, b):
    a, b = lift(a), lift(b)
    return mk("minimum", [a, b], _bshape([a, b]))


def conv2d(x, w, stride, padding):
    """``tf.nn.conv2d(x, w, [1, s, s, 1], padding)``, NHWC x HWIO; output shape as TF's SAME."""
    x, w = lift(x), lift(w)
    if padding != "SAME":
        raise NotImplementedError(padding)
    n, h, wd, _ = x.shape
    return mk("conv", [x, w, int(stride), padding], (n, -(-h // stride), -(-wd // stride), w.shape[-1]))


def max_pool(x, k, s, padding):
    x = lift(x)
    n, h, w, c = x.shape
    return mk("maxpool", [x, int(k), int(s), padding], (n, -(-h // s), -(-w // s), c))


def flatten(x):
    n = x.shape[0]
    return mk("flatten", [x], (n, int(np.prod(x.shape[1:]))))


def var(name, shape):
    """a model variable, by its TF name below the model's outer scope (``conv_1/conv_1_filters``)"""
    return Sym("var", [name], shape)


def inp(name, shape):
    return Sym("in", [name], shape)


# ---------------------------------------------------------------------------------------------
def render(x, depth=6):
    """readable s-expression (cut at ``depth``); operands of +/* in canonical order"""
    if not isinstance(x, Sym):
        return repr(x)
    if x.op == "c":
        return f"{x.args[0]:g}"
    if x.op in ("var", "in"):
        return x.args[0]
    if depth <= 0:
        return f"<{x.op}:{x.h[:8]}>"
    inner = ", ".join(render(a, depth - 1) for a in x.args)
    return f"{x.op}({inner})"


def free_inputs(x, seen=None):
    """names of the ``in`` leaves the expression depends on"""
    seen = set() if seen is None else seen
    out = set()
    stack = [x]
    while stack:
        s = stack.pop()
        if not isinstance(s, Sym) or s.h in seen:
            continue
        seen.add(s.h)
        if s.op == "in":
            out.add(s.args[0])
        stack.extend(a for a in s.args if isinstance(a, Sym))
        for a in s.args:
            if isinstance(a, tuple):
                stack.extend(e for e in a if isinstance(e, Sym))
    return out


def node_count(x):
    seen, stack = set(), [x]
    while stack:
        s = stack.pop()
        if not isinstance(s, Sym) or s.h in seen:
            continue
        seen.add(s.h)
        stack.extend(a for a in s.args if isinstance(a, Sym))
    return len(seen)
