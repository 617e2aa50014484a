"""Dev tool (build container only: /root/reference does not exist on the GPU box).

Evaluates the reference's hGRU code symbolically, straight from its source text:

* ``hgru_module.auxilliary_variables`` and ``ContextualCircuit.__init__`` / ``prepare_tensors`` /
  ``build`` / ``full`` / ``circuit_input`` / ``circuit_output`` / ``process_p`` /
  ``p_convolution`` / ``conv_2d_op`` / ``input_integration`` / ``output_integration`` and the
  rest of the class (``/root/reference/hgru_module.py:9-959``);
* ``hgru_pose.model.__init__`` / ``build`` / ``hgru_layer`` / ``conv_layer`` / ``fc_layer`` /
  ``max_pool`` / ``get_*_var`` (``/root/reference/hgru_pose.py:8-216``).

The files are Python 2 and TensorFlow 1 and cannot be imported; every method body
is parsed on its own as an AST (the one Python-2 ``print`` statement, ``hgru_module.py:295``,
becomes ``pass``) and run by a small interpreter whose ``tf`` builds ``tests/symbolic.py`` nodes
instead of graph ops.  Control flow (the aux-flag branches, ``tf.while_loop``, which is unrolled
with its integer counter) is evaluated for real, so the expression that comes out is the one the
reference's own code builds for the given aux.  ``tests/test_hgru_structure.py`` compares it with
the oracle's (``oracle/hgru_ref.py``) by Merkle hash.

Reference defects are resolved at exactly the point the reference hits them, each
recorded in ``Interp.defects``:
  1. ``utils.py_utils`` missing        -> ``ifloor`` / ``iceil`` = ``int(floor/ceil)``
     ``ops.initialization`` missing    -> ``xavier_initializer`` = a fresh random tensor
                                          (an input named ``rand#k``, k = call order)
  3. ``hgru_layer`` returns a tuple    -> batch_normalization consumes element 0 (``O``)
  4. ``self.relu3`` undefined (104)    -> ``self.relu1``
  5. BN ``axis=3`` on a rank-2 tensor  -> per-feature BN over the last axis

    python tools/extract_hgru.py            # prints the one-step update rule and digests
"""
from __future__ import annotations

import ast
import math
import os
import re
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import symbolic as S  # noqa: E402

REF_DIR = "/root/reference"
REF_MODULE = os.path.join(REF_DIR, "hgru_module.py")
REF_POSE = os.path.join(REF_DIR, "hgru_pose.py")


# ---------------------------------------------------------------------------------------------
# source -> per-function ASTs
# ---------------------------------------------------------------------------------------------
def _py2_fix(line):
    # Python-2 print statement (hgru_module.py:295) -> no-op; print(...) calls stay calls
    return re.sub(r"^(\s*)print\s+['\"].*$", r"\1pass", line)


def _functions(path, classname=None):
    """{name: (ast.FunctionDef, first line number)} of the module-level defs, or of one class"""
    lines = open(path).read().split("\n")
    if classname is None:
        indent, lo, hi = "", 0, len(lines)
    else:
        lo = next(i for i, l in enumerate(lines) if re.match(rf"class {classname}\b", l)) + 1
        hi = next((i for i in range(lo, len(lines)) if re.match(r"\S", lines[i])), len(lines))
        indent = "    "
    out = {}
    i = lo
    while i < hi:
        m = re.match(rf"^{indent}def (\w+)\(", lines[i])
        if not m:
            i += 1
            continue
        j = i + 1
        while j < hi and not re.match(rf"^{indent}\S", lines[j]):
            j += 1
        body = "\n".join(_py2_fix(l[len(indent):]) for l in lines[i:j])
        out[m.group(1)] = (ast.parse(body).body[0], i + 1)
        i = j
    return out


# ---------------------------------------------------------------------------------------------
# interpreter
# ---------------------------------------------------------------------------------------------
class _Return(Exception):
    def __init__(self, v):
        self.v = v


class Obj:
    """an instance of an interpreted class"""

    def __init__(self, cls):
        object.__setattr__(self, "_cls", cls)
        object.__setattr__(self, "_attrs", {})

    def get(self, name, interp):
        if name in self._attrs:
            return self._attrs[name]
        if name in self._cls.methods:
            return Method(self._cls.methods[name], self, interp, self._cls)
        return interp.missing_attr(self, name)

    def set(self, name, v):
        self._attrs[name] = v

    def has(self, name):
        return name in self._attrs or name in self._cls.methods


class Cls:
    def __init__(self, name, methods, interp, globs):
        self.name, self.methods, self.interp, self.globs = name, methods, interp, globs

    def __call__(self, *args, **kw):
        o = Obj(self)
        if "__init__" in self.methods:
            Method(self.methods["__init__"], o, self.interp, self)(*args, **kw)
        return o


class Method:
    def __init__(self, fn, bound, interp, cls):
        self.fn, self.bound, self.interp, self.cls = fn, bound, interp, cls

    def __call__(self, *args, **kw):
        fdef, _ = self.fn
        return self.interp.call(fdef, self.cls.globs, ((self.bound,) if self.bound is not None else ()) + args, kw)


class Func:
    def __init__(self, fn, interp, globs):
        self.fn, self.interp, self.globs = fn, interp, globs

    def __call__(self, *args, **kw):
        return self.interp.call(self.fn[0], self.globs, args, kw)


class NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class Interp:
    def __init__(self):
        self.defects = []
        self.scope = []
        self.rand_count = 0
        self.bn_count = 0
        self.weights = {}

    # -- resolutions at the point of the defect ---------------------------------------------
    def missing_attr(self, obj, name):
        if obj._cls.name == "model" and name == "relu3":
            self.defects.append("4: self.relu3 undefined -> self.relu1 (hgru_pose.py:104)")
            return obj.get("relu1", self)
        raise AttributeError(f"{obj._cls.name}.{name}")

    # -- function calls ---------------------------------------------------------------------
    def call(self, fdef, globs, args, kw):
        env = {}
        a = fdef.args
        names = [x.arg for x in a.args]
        defaults = [self.expr(d, globs, {}) for d in a.defaults]
        dmap = dict(zip(names[len(names) - len(defaults):], defaults))
        if len(args) > len(names):
            raise TypeError(f"{fdef.name}: too many arguments")
        for n, v in zip(names, args):
            env[n] = v
        for k, v in kw.items():
            if k not in names or k in env:
                raise TypeError(f"{fdef.name}: bad keyword {k}")
            env[k] = v
        for n in names:
            if n not in env:
                if n not in dmap:
                    raise TypeError(f"{fdef.name}: missing {n}")
                env[n] = dmap[n]
        try:
            self.block(fdef.body, globs, env)
        except _Return as r:
            return r.v
        return None

    # -- statements -------------------------------------------------------------------------
    def block(self, body, g, env):
        for st in body:
            self.stmt(st, g, env)

    def assign(self, tgt, v, g, env):
        if isinstance(tgt, ast.Name):
            env[tgt.id] = v
        elif isinstance(tgt, ast.Attribute):
            o = self.expr(tgt.value, g, env)
            if isinstance(o, Obj):
                o.set(tgt.attr, v)
            else:
                setattr(o, tgt.attr, v)
        elif isinstance(tgt, ast.Subscript):
            o = self.expr(tgt.value, g, env)
            o[self.expr(tgt.slice, g, env)] = v
        elif isinstance(tgt, (ast.Tuple, ast.List)):
            vs = list(v)
            if len(vs) != len(tgt.elts):
                raise ValueError("unpack mismatch")
            for t, x in zip(tgt.elts, vs):
                self.assign(t, x, g, env)
        else:
            raise NotImplementedError(ast.dump(tgt))

    def stmt(self, st, g, env):
        if isinstance(st, ast.Expr):
            self.expr(st.value, g, env)
        elif isinstance(st, ast.Pass):
            pass
        elif isinstance(st, ast.Assign):
            v = self.expr(st.value, g, env)
            for t in st.targets:
                self.assign(t, v, g, env)
        elif isinstance(st, ast.AugAssign):
            # tensors are immutable: `O *= g` builds a new tensor and rebinds the target
            cur = self.expr(st.target, g, env)
            v = self.binop(st.op, cur, self.expr(st.value, g, env))
            self.assign(st.target, v, g, env)
        elif isinstance(st, ast.If):
            c = self.expr(st.test, g, env)
            if not isinstance(c, (bool, int, type(None), str, list, dict, tuple, float)):
                raise TypeError(f"data-dependent branch at line {st.lineno}")
            self.block(st.body if c else st.orelse, g, env)
        elif isinstance(st, ast.For):
            for v in list(self.expr(st.iter, g, env)):
                self.assign(st.target, v, g, env)
                self.block(st.body, g, env)
        elif isinstance(st, ast.Return):
            raise _Return(self.expr(st.value, g, env) if st.value is not None else None)
        elif isinstance(st, ast.With):
            ctxs = [self.expr(it.context_expr, g, env) for it in st.items]
            for c in ctxs:
                c.__enter__()
            try:
                self.block(st.body, g, env)
            finally:
                for c in reversed(ctxs):
                    c.__exit__(None, None, None)
        elif isinstance(st, ast.Raise):
            raise RuntimeError(f"reference raises at line {st.lineno}: {ast.unparse(st)}")
        else:
            raise NotImplementedError(ast.dump(st))

    # -- expressions ------------------------------------------------------------------------
    def binop(self, op, a, b):
        if isinstance(op, ast.Add):
            return a + b
        if isinstance(op, ast.Sub):
            return a - b
        if isinstance(op, ast.Mult):
            return a * b
        if isinstance(op, ast.Div):
            if isinstance(a, int) and isinstance(b, int):
                return a // b      # Python 2 integer division
            return a / b
        if isinstance(op, ast.FloorDiv):
            return a // b
        if isinstance(op, ast.Mod):
            return a % b
        raise NotImplementedError(ast.dump(op))

    def expr(self, e, g, env):
        if isinstance(e, ast.Constant):
            return e.value
        if isinstance(e, ast.Name):
            if e.id in env:
                return env[e.id]
            if e.id in g:
                return g[e.id]
            raise NameError(e.id)
        if isinstance(e, ast.Attribute):
            o = self.expr(e.value, g, env)
            if isinstance(o, Obj):
                return o.get(e.attr, self)
            if isinstance(o, dict) and e.attr == "iteritems":
                return o.items
            return getattr(o, e.attr)
        if isinstance(e, ast.Subscript):
            o = self.expr(e.value, g, env)
            k = self.expr(e.slice, g, env)
            if isinstance(o, Obj):
                return o.get(k, self)        # __getitem__ = getattr (hgru_module.py:55-56)
            return o[k]
        if isinstance(e, ast.Slice):
            return slice(*(self.expr(x, g, env) if x is not None else None for x in (e.lower, e.upper, e.step)))
        if isinstance(e, ast.Call):
            f = self.expr(e.func, g, env)
            args = []
            for a in e.args:
                if isinstance(a, ast.Starred):
                    args.extend(self.expr(a.value, g, env))
                else:
                    args.append(self.expr(a, g, env))
            kw = {}
            for k in e.keywords:
                if k.arg is None:
                    kw.update(self.expr(k.value, g, env))
                else:
                    kw[k.arg] = self.expr(k.value, g, env)
            return f(*args, **kw)
        if isinstance(e, ast.BinOp):
            return self.binop(e.op, self.expr(e.left, g, env), self.expr(e.right, g, env))
        if isinstance(e, ast.UnaryOp):
            v = self.expr(e.operand, g, env)
            if isinstance(e.op, ast.USub):
                return -v
            if isinstance(e.op, ast.Not):
                return not v
            raise NotImplementedError(ast.dump(e.op))
        if isinstance(e, ast.BoolOp):
            if isinstance(e.op, ast.And):
                v = True
                for x in e.values:
                    v = self.expr(x, g, env)
                    if not v:
                        return v
                return v
            v = False
            for x in e.values:
                v = self.expr(x, g, env)
                if v:
                    return v
            return v
        if isinstance(e, ast.Compare):
            left = self.expr(e.left, g, env)
            for op, rn in zip(e.ops, e.comparators):
                right = self.expr(rn, g, env)
                ok = {ast.Eq: lambda a, b: a == b, ast.NotEq: lambda a, b: a != b,
                      ast.Lt: lambda a, b: a < b, ast.LtE: lambda a, b: a <= b,
                      ast.Gt: lambda a, b: a > b, ast.GtE: lambda a, b: a >= b,
                      ast.Is: lambda a, b: a is b, ast.IsNot: lambda a, b: a is not b,
                      ast.In: lambda a, b: a in b, ast.NotIn: lambda a, b: a not in b}[type(op)](left, right)
                if isinstance(ok, S.Sym):
                    raise TypeError("symbolic comparison")
                if not ok:
                    return False
                left = right
            return True
        if isinstance(e, ast.List):
            return [self.expr(x, g, env) for x in e.elts]
        if isinstance(e, ast.Tuple):
            return tuple(self.expr(x, g, env) for x in e.elts)
        if isinstance(e, ast.Dict):
            return {self.expr(k, g, env): self.expr(v, g, env) for k, v in zip(e.keys, e.values)}
        if isinstance(e, ast.ListComp):
            if len(e.generators) != 1 or e.generators[0].ifs:
                raise NotImplementedError("comprehension")
            gen = e.generators[0]
            out = []
            for v in list(self.expr(gen.iter, g, env)):
                inner = dict(env)
                self.assign(gen.target, v, g, inner)
                out.append(self.expr(e.elt, g, inner))
            return out
        if isinstance(e, ast.Lambda):
            raise NotImplementedError("lambda")
        raise NotImplementedError(ast.dump(e))


# ---------------------------------------------------------------------------------------------
# TensorFlow 1 stand-in: graph ops become symbolic nodes (semantics as documented for TF 1.x)
# ---------------------------------------------------------------------------------------------
class _Shape(list):
    def as_list(self):
        return list(self)


class _Init:
    """an initializer expression: only its shape matters (values are never part of the graph)"""

    def __init__(self, shape):
        self.shape = None if shape is None else tuple(int(s) for s in shape)

    def __neg__(self):
        return self


def _sym_shape(x):
    return _Shape([int(s) for s in x.shape])


class _TensorArray:
    def __init__(self, dtype, size):
        self.items = [None] * size

    def write(self, i, v):
        self.items[i] = v
        return self

    def stack(self):
        return S.mk("stack", [tuple(self.items)], (len(self.items),) + tuple(self.items[0].shape))


def make_tf(interp: Interp):
    def scoped(name):
        return "/".join(interp.scope + [name])

    class VarScope:
        def __init__(self, name):
            self.name = name

        def __enter__(self):
            interp.scope.append(self.name)

        def __exit__(self, *a):
            interp.scope.pop()

    def get_variable(name, dtype=None, initializer=None, trainable=True, shape=None):
        full = scoped(name)
        if shape is None:
            if isinstance(initializer, _Init):
                shape = initializer.shape
            elif isinstance(initializer, np.ndarray):
                shape = initializer.shape
            elif isinstance(initializer, S.Sym):
                shape = initializer.shape
        if full in interp.weights:
            raise ValueError(f"variable {full} created twice")
        v = S.var(full, shape)
        interp.weights[full] = tuple(shape) if shape is not None else None
        return v

    def constant(value, dtype=None, name=None):
        if isinstance(value, bool) or isinstance(value, int):
            return value        # an integer scalar (the while_loop counter): kept concrete
        if isinstance(value, float):
            return S.const(value)
        raise NotImplementedError("tf.constant of an array")

    def conv2d(data, weights, strides, padding):
        assert strides[0] == strides[3] == 1 and strides[1] == strides[2], strides
        return S.conv2d(data, weights, strides[1], padding)

    def max_pool(x, ksize, strides, padding, name=None):
        assert ksize[1] == ksize[2] and strides[1] == strides[2] and ksize[0] == ksize[3] == 1
        return S.max_pool(x, ksize[1], strides[1], padding)

    def batch_normalization(inputs, axis=-1, momentum=0.99, epsilon=1e-3, center=True, scale=True,
                            training=False, fused=None, name=None):
        if training:
            raise RuntimeError("training-mode batch statistics")
        if isinstance(inputs, tuple):
            interp.defects.append("3: batch_normalization of the hgru_layer tuple -> its element 0 (O)")
            inputs = inputs[0]
        if axis not in (-1, len(inputs.shape) - 1):
            interp.defects.append(f"5: BN axis={axis} on a rank-{len(inputs.shape)} tensor -> last axis")
        if not (center and scale):
            raise NotImplementedError("BN without center/scale")
        nm = "batch_normalization" + (f"_{interp.bn_count}" if interp.bn_count else "")
        interp.bn_count += 1
        c = inputs.shape[-1]
        g = get_variable(nm + "/gamma", shape=(c,))
        b = get_variable(nm + "/beta", shape=(c,))
        m = get_variable(nm + "/moving_mean", shape=(c,))
        v = get_variable(nm + "/moving_variance", shape=(c,))
        # inference FusedBatchNorm: gamma * (x - mean) / sqrt(var + eps) + beta
        return g * (inputs - m) / S.power(v + float(epsilon), 0.5) + b

    def reshape(x, shape):
        if len(shape) == 2 and shape[0] == -1 and shape[1] == int(np.prod(x.shape[1:])):
            return S.flatten(x)
        raise NotImplementedError(f"reshape {x.shape} -> {shape}")

    def while_loop(cond, body, loop_vars, back_prop=True, swap_memory=False):
        vs = list(loop_vars)
        for _ in range(10000):
            c = cond(*vs)
            if not isinstance(c, bool):
                raise TypeError("while_loop condition must be concrete")
            if not c:
                return vs
            vs = list(body(*vs))
        raise RuntimeError("while_loop did not terminate")

    def zeros_like(x):
        return S.const(0.0, x.shape)

    def identity(x, name=None):
        return x

    def gather(params, idx, axis=None):
        assert axis in (None, -1, 0)
        return S.mk("gather", [params, idx], ())

    def transpose(x, perm, name=None):
        shape = tuple(x.shape[p] for p in perm)
        return S.mk("transpose", [x, tuple(perm)], shape)

    nn = types.SimpleNamespace(
        conv2d=conv2d, bias_add=lambda x, b: S.add(x, b), relu=S.relu, tanh=S.tanh, sigmoid=S.sigmoid,
        max_pool=max_pool, dropout=None, atrous_conv2d=None)
    tf = types.SimpleNamespace(
        nn=nn, layers=types.SimpleNamespace(batch_normalization=batch_normalization),
        float32="float32", constant=constant, get_variable=get_variable, variable_scope=VarScope,
        get_default_graph=lambda: types.SimpleNamespace(gradient_override_map=lambda m: NullCtx()),
        while_loop=while_loop, zeros_like=zeros_like, identity=identity, gather=gather,
        transpose=transpose, TensorArray=_TensorArray, reshape=reshape, matmul=lambda a, b: a @ b,
        minimum=S.minimum, maximum=S.maximum, sigmoid=S.sigmoid, tanh=S.tanh,
        log=lambda x: x, random_uniform=lambda shape, minval=0, maxval=1: _Init(shape),
        ones=lambda shape, dtype=None: _Init(shape if isinstance(shape, (list, tuple)) else [shape]),
        contrib=types.SimpleNamespace(layers=types.SimpleNamespace(
            xavier_initializer=lambda uniform=True: _Init(None),
            xavier_initializer_conv2d=lambda uniform=True: _Init(None))),
        truncated_normal=lambda shape, mean=0.0, stddev=1.0: _Init(shape))
    return tf


def make_globals(interp: Interp):
    tf = make_tf(interp)

    def ifloor(x):
        return int(math.floor(x))

    def iceil(x):
        return int(math.ceil(x))

    def xavier_initializer(shape, uniform=True, mask=None):
        # DEFECT 1 (ops.initialization missing): a fresh random tensor of `shape`; used either as a
        # variable's initializer (value irrelevant) or, for hidden_init='random', as the state itself
        k = interp.rand_count
        interp.rand_count += 1
        return S.inp(f"rand#{k}", tuple(int(s) for s in shape))

    interp.defects.append("1: utils.py_utils / ops.initialization missing -> int(floor/ceil), fresh random tensor")
    g = {
        "tf": tf, "np": np, "basestring": str, "isinstance": isinstance, "int": int, "float": float,
        "len": len, "range": range, "list": list, "dict": dict, "setattr": lambda o, k, v: o.set(k, v),
        "hasattr": lambda o, k: o.has(k), "getattr": lambda o, k: o.get(k, interp), "print": lambda *a, **k: None,
        "NotImplementedError": NotImplementedError, "RuntimeError": RuntimeError, "True": True,
        "False": False, "None": None, "object": object, "type": type,
        "py_utils": types.SimpleNamespace(ifloor=ifloor, iceil=iceil),
        "initialization": types.SimpleNamespace(xavier_initializer=xavier_initializer),
    }
    return g


def _patch_shapes(g):
    """give Sym inputs a TF-like ``get_shape()`` for the reference's static shape reads"""
    S.Sym.get_shape = lambda self: _sym_shape(self)

    def set_shape(self, shape):
        if [int(x) for x in shape] != list(self.shape):
            raise ValueError(f"set_shape {shape} on {self.shape}")
    S.Sym.set_shape = set_shape


def load(interp=None):
    interp = interp or Interp()
    g = make_globals(interp)
    _patch_shapes(g)
    mod_fns = _functions(REF_MODULE)
    g["auxilliary_variables"] = Func(mod_fns["auxilliary_variables"], interp, g)
    cc = Cls("ContextualCircuit", _functions(REF_MODULE, "ContextualCircuit"), interp, g)
    g_pose = dict(g)
    g_pose["hgru_module"] = types.SimpleNamespace(ContextualCircuit=cc)
    model = Cls("model", _functions(REF_POSE, "model"), interp, g_pose)
    return interp, cc, model


# ---------------------------------------------------------------------------------------------
# the expressions the tests compare
# ---------------------------------------------------------------------------------------------
def pose_aux():
    """hgru_pose.model().aux, read from the reference (hgru_pose.py:20-39)"""
    _, _, model = load()
    return dict(model().get("aux", None))


def circuit(n, h, w, ssf, timesteps, hidden_init="random", store_states=False):
    """ContextualCircuit(X, timesteps, SRF=1, SSN=15, SSF=ssf, aux=hgru_pose aux + overrides).build()
    with X an input named 'X'; returns (interp, O, weights-dict)"""
    interp, cc, model = load()
    aux = dict(model().get("aux", interp))
    aux["hidden_init"] = hidden_init
    aux["store_states"] = store_states
    X = S.inp("X", (n, h, w, 64))
    c = cc(X=X, timesteps=timesteps, SRF=1, SSN=15, SSF=ssf, strides=[1, 1, 1, 1], padding="SAME", aux=aux)
    res = c.get("build", interp)()
    return interp, res, c


def pose(n, crop, output_shape=69):
    """hgru_pose.model().build(depth, output_shape) with depth an input named 'depth'"""
    interp, _, model = load()
    m = model()
    depth = S.inp("depth", (n, crop, crop, 1))
    m.get("build", interp)(depth, output_shape)
    return interp, m


if __name__ == "__main__":
    it, res, c = circuit(2, 16, 32, 15, 2)
    O = res[0]
    print("defects:", it.defects)
    print("weights:", sorted(it.weights))
    print("free inputs of O_T:", sorted(S.free_inputs(O)), "nodes", S.node_count(O))
    it1, res1, _ = circuit(2, 16, 32, 15, 1)
    print("one step O_1 =", S.render(res1[0], 12))
    it2, m = pose(2, 128)
    out = m.get("out_put", it2)
    print("pose defects:", it2.defects)
    print("pose out_put nodes", S.node_count(out), "free", sorted(S.free_inputs(out)), out.shape)
