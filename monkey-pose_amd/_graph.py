"""Graph recording for the layer-graph runtime (``MP_MODEL_GRAPH``, ``mp_graph_set`` /
``mp_graph_fwd`` in include/monkeypose.h).

The reference's regressors are TF1 graph builders: ``build()`` chains ``conv_layer``,
``max_pool``, ``tf.concat``, ``fc_layer``, ``tf.nn.relu`` and ``tf.identity`` calls and TF runs
the graph later.  ``GraphRecorder`` keeps that split: the facade's ``build()`` makes the same calls
on symbolic tensors (``Sym``, shape-checked as TF's graph construction would be), and the recorded
op list goes to the native runtime, which plans concat placement, streams and a hipGraph once and
replays it per forward.  Helpers restated: conv_layer / max_pool / avg_pool / max_pool_4 /
fc_layer of train_dense_hier_networks.py:2416-2455.
"""
from __future__ import annotations

import ctypes
import hashlib
import json
from typing import Dict, List, Optional, Sequence

from . import _lib

MP_OP_CONV, MP_OP_MAXPOOL, MP_OP_AVGPOOL, MP_OP_CONCAT, MP_OP_FC, MP_OP_RELU, MP_OP_IDENTITY = range(1, 8)
MAX_SRC = 8
_KIND_NAME = {MP_OP_CONV: "conv", MP_OP_MAXPOOL: "maxpool", MP_OP_AVGPOOL: "avgpool",
              MP_OP_CONCAT: "concat", MP_OP_FC: "fc", MP_OP_RELU: "relu", MP_OP_IDENTITY: "identity"}


class GraphOp(ctypes.Structure):
    """``mp_graph_op`` (include/monkeypose.h)."""
    _fields_ = [("kind", ctypes.c_int32), ("out", ctypes.c_int32), ("n_src", ctypes.c_int32),
                ("src", ctypes.c_int32 * MAX_SRC), ("ksize", ctypes.c_int32),
                ("stride", ctypes.c_int32), ("cout", ctypes.c_int32), ("name", ctypes.c_char_p)]


class Sym:
    """A symbolic NHWC tensor ([n, H, W, C], or [n, C] after fc_layer) of a recorded graph."""

    def __init__(self, g: "GraphRecorder", tid: int, shape: Sequence[int]):
        self.graph, self.id, self.shape = g, tid, tuple(int(s) for s in shape)
        self.label: Optional[str] = None

    def get_shape(self):
        return [None] + list(self.shape)

    @property
    def channels(self) -> int:
        return self.shape[-1]

    def __repr__(self):
        return f"Sym({self.label or self.id}, {list(self.shape)})"


def _same(n: int, s: int) -> int:
    return -(-n // s)


class GraphRecorder:
    def __init__(self, h: int, w: int, c: int = 1):
        self.ops: List[dict] = []
        self.input = Sym(self, 0, (h, w, c))
        self.input.label = "lr_input"
        self._next = 1

    def _new(self, shape) -> Sym:
        s = Sym(self, self._next, shape)
        self._next += 1
        return s

    def _add(self, kind, out: Sym, srcs: Sequence[Sym], **kw) -> Sym:
        for s in srcs:
            if s.graph is not self:
                raise ValueError("tensor from another graph")
        self.ops.append(dict(kind=kind, out=out, srcs=list(srcs), **kw))
        return out

    # conv_layer (2431-2446): relu(conv2d(x, W[k,k,cin,cout], stride, SAME) + b)
    def conv(self, x: Sym, cin: int, cout: int, name: str, k: int = 3, stride: int = 1) -> Sym:
        if len(x.shape) != 3:
            raise ValueError(f"conv {name}: input must be NHWC")
        if int(cin) != x.channels:   # TF raises at conv2d construction on a channel mismatch
            raise ValueError(f"conv {name}: in_channels {cin} != input channels {x.channels}")
        h, w, _ = x.shape
        return self._add(MP_OP_CONV, self._new((_same(h, stride), _same(w, stride), int(cout))), [x],
                         name=name, k=int(k), stride=int(stride), cin=int(cin), cout=int(cout))

    # max_pool (2426-2429) / max_pool_4 (2421-2424) / avg_pool (2416-2419), SAME
    def pool(self, x: Sym, k: int = 2, avg: bool = False) -> Sym:
        h, w, c = x.shape
        return self._add(MP_OP_AVGPOOL if avg else MP_OP_MAXPOOL, self._new((_same(h, k), _same(w, k), c)),
                         [x], k=int(k))

    def concat(self, xs: Sequence[Sym]) -> Sym:
        if not 1 <= len(xs) <= MAX_SRC:
            raise ValueError(f"tf.concat of {len(xs)} tensors (1..{MAX_SRC} supported)")
        if len({x.shape[:-1] for x in xs}) != 1:
            raise ValueError("tf.concat: spatial shapes differ")
        return self._add(MP_OP_CONCAT, self._new(xs[0].shape[:-1] + (sum(x.channels for x in xs),)), xs)

    # fc_layer (2448-2455): reshape(x, [-1, in_size]) @ W + b
    def fc(self, x: Sym, in_size: int, out_size: int, name: str) -> Sym:
        flat = 1
        for s in x.shape:
            flat *= s
        if int(in_size) != flat:
            raise ValueError(f"fc {name}: in_size {in_size} != flattened input {flat}")
        return self._add(MP_OP_FC, self._new((int(out_size),)), [x], name=name, cin=flat,
                         cout=int(out_size))

    def relu(self, x: Sym) -> Sym:
        return self._add(MP_OP_RELU, self._new(x.shape), [x])

    def identity(self, x: Sym) -> Sym:
        return self._add(MP_OP_IDENTITY, self._new(x.shape), [x])

    # ---- export ----
    def records(self) -> List[dict]:
        """The op list in the schema of tools/extract_dense_hier.py (labels = the reference's
        attribute names), for structural comparison with the reference."""
        out = []
        for o in self.ops:
            r = dict(op=_KIND_NAME[o["kind"]], out=o["out"].label or f"t{o['out'].id}")
            labels = [s.label or f"t{s.id}" for s in o["srcs"]]
            if o["kind"] == MP_OP_CONCAT:
                r["srcs"] = labels
            else:
                r["src"] = labels[0]
            for k in ("name", "k", "stride", "cin", "cout"):
                if k in o:
                    r[k] = o[k]
            out.append(r)
        return out

    def layers(self) -> List[dict]:
        return [o for o in self.ops if o["kind"] in (MP_OP_CONV, MP_OP_FC)]

    def to_c(self):
        arr = (GraphOp * len(self.ops))()
        keep = []
        for i, o in enumerate(self.ops):
            e = arr[i]
            e.kind, e.out, e.n_src = o["kind"], o["out"].id, len(o["srcs"])
            for j, s in enumerate(o["srcs"]):
                e.src[j] = s.id
            e.ksize = o.get("k", 0)
            e.stride = o.get("stride", 1)
            e.cout = o.get("cout", 0)
            if "name" in o:
                b = o["name"].encode()
                keep.append(b)
                e.name = b
        return arr, keep


def canonical_digest(records: List[dict]) -> str:
    """sha256 of the op list with line numbers dropped (the structural fingerprint committed in
    tests/golden/dense_hier_graph_digest.json)."""
    keys = ("op", "out", "src", "srcs", "name", "k", "stride", "cin", "cout")
    canon = [{k: r[k] for k in keys if k in r} for r in records]
    return hashlib.sha256(json.dumps(canon, sort_keys=True).encode()).hexdigest()


def install(ctx: "_lib.Context", g: GraphRecorder, outputs: Sequence[Sym]) -> None:
    arr, keep = g.to_c()
    outs = (ctypes.c_int32 * len(outputs))(*[o.id for o in outputs])
    _lib.check(ctx.lib.mp_graph_set(ctx.h, arr, len(g.ops), g.input.channels, outs, len(outputs)))
    del keep


def layer_shapes(g: GraphRecorder) -> Dict[str, tuple]:
    """{layer scope: weight shape} for every conv (HWIO) and fc ([in, out]) of the graph."""
    d = {}
    for o in g.layers():
        d[o["name"]] = ((o["k"], o["k"], o["cin"], o["cout"]) if o["kind"] == MP_OP_CONV
                        else (o["cin"], o["cout"]))
    return d


def flops_per_sample(g: GraphRecorder) -> float:
    """Algorithmic FLOPs of one sample: 2 * Ho * Wo * k * k * cin * cout per conv, 2 * K * N per fc."""
    t = 0.0
    for o in g.layers():
        if o["kind"] == MP_OP_CONV:
            ho, wo, _ = o["out"].shape
            t += 2.0 * ho * wo * o["k"] * o["k"] * o["cin"] * o["cout"]
        else:
            t += 2.0 * o["cin"] * o["cout"]
    return t
