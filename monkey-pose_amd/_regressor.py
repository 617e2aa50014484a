"""Shared machinery of the dense / hierarchical regressor facades (weights, context, checks)."""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

from . import _lib
from . import weights as W


class RegressorBase:
    MODEL_KIND = 0

    def __init__(self, trainable=True):
        self.trainable = trainable
        self.data_dict = None           # {layer: [W, b]} as in get_var
        self.var_dict = {}
        self.weights: Optional[Dict[str, np.ndarray]] = None
        self.weight_seed = 1234
        # conv / fc precision: 'auto' (= 'fp32_split': fp32-accurate f16x3 MFMA, the fastest
        # fp32-class path) or 'fp32' (exact fp32 MFMA)
        self.compute_dtype = 'auto'
        self._ctx: Optional[_lib.Context] = None
        self._ctx_key = None

    def __getitem__(self, name):
        return getattr(self, name)

    def __contains__(self, name):
        return hasattr(self, name)

    def load_weights(self, weights: Dict[str, np.ndarray], synthesize_missing: bool = False) -> None:
        """Variables keyed by TF name (``cnn/...``).  Like ``saver.restore`` of a checkpoint
        (train_cnn_networks_hgru.py:248-250), every variable the model needs must be present:
        build() raises ``KeyError`` naming the missing ones, unless ``synthesize_missing=True``
        fills them with the seeded stand-in initialisers (``weights.synth_value``).  A model with
        no weights loaded at all runs on those stand-ins, as the reference runs on its
        initialisers."""
        self.weights = {(k if k.startswith("cnn/") else "cnn/" + k): v for k, v in weights.items()}
        self._ctx_key = None
        self._strict = not synthesize_missing

    def load_checkpoint(self, path: str, remap=None, strict: bool = True) -> None:
        """Weights from a TF1 V2 checkpoint (see ``hgru_pose.model.load_checkpoint``)."""
        from . import tf_checkpoint as C
        t = C.model_variables(C.read_checkpoint(path))
        self.load_weights(remap(t) if remap else t, synthesize_missing=not strict)

    def load_npz(self, path: str, synthesize_missing: bool = False) -> None:
        with np.load(path, allow_pickle=False) as z:
            self.load_weights({k: z[k] for k in z.files}, synthesize_missing)

    def _on_context(self, ctx: _lib.Context) -> None:
        """hook between mp_create and the weights of an MP_MODEL_GRAPH context (installs its graph)"""

    def _table(self, **kw) -> List[W.Var]:
        raise NotImplementedError

    def _resolve(self, table) -> Dict[str, np.ndarray]:
        given = dict(self.weights or {})
        covered = set()
        for layer in (self.data_dict or {}):
            covered |= {f"cnn/{layer}/{layer}{s}" for s in ("_weights", "_biases", "_filters")}
        missing = [v.name for v in table if v.name not in given and v.name not in covered]
        if missing and self.weights is not None and getattr(self, "_strict", True):
            raise KeyError(f"the loaded weights lack {len(missing)} variable(s) the model needs "
                           f"(load_weights(..., synthesize_missing=True) fills them): {missing[:8]}")
        out = {v.name: (np.asarray(given[v.name], np.float32) if v.name in given
                        else W.synth_value(v, self.weight_seed)) for v in table}
        if self.data_dict is not None:
            for layer, vals in self.data_dict.items():
                suff = ("_weights", "_biases") if "fc" in layer else ("_filters", "_biases")
                for idx in (0, 1):
                    out[f"cnn/{layer}/{layer}{suff[idx]}"] = np.asarray(vals[idx], np.float32)
        for k, v in out.items():
            self.var_dict[(k.split("/")[1], k)] = v
        return out

    def _dtype(self) -> str:
        dt = {'auto': 'fp32_split', 'fp32_split': 'fp32_split', 'f32_split': 'fp32_split',
              'fp32': 'fp32', 'f32': 'fp32', 'bf16': 'bf16'}.get(self.compute_dtype)
        if dt is None:
            raise ValueError(f"regressor compute_dtype must be 'auto', 'fp32_split', 'fp32' or 'bf16', "
                             f"got {self.compute_dtype!r}")
        return dt

    def _context(self, key, table, device: int, kind: Optional[int] = None) -> _lib.Context:
        dt = self._dtype()
        kind = self.MODEL_KIND if kind is None else kind
        key = (key, kind, device, id(self.weights), id(self.data_dict), dt)
        if self._ctx is None or self._ctx_key != key:
            ctx = _lib.Context(kind, device)
            if kind == _lib.MP_MODEL_GRAPH:
                self._on_context(ctx)
            for name, val in self._resolve(table).items():
                ctx.set_weight(name, val)
            ctx.finalize(_lib.dtype_code(dt))
            self._ctx, self._ctx_key = ctx, key
        return self._ctx

    @staticmethod
    def _check_input(depth, batch_norm, train_mode):
        import torch
        if train_mode:
            raise NotImplementedError("train_mode=True (dropout / backward) is outside the inference path")
        if batch_norm is not None:
            raise NotImplementedError("conv_layer batchnorm= (batch-moment BN) is a training option")
        if not isinstance(depth, torch.Tensor) or not depth.is_cuda:
            raise TypeError("depth must be a CUDA (ROCm) torch tensor")
        if depth.dim() != 4 or depth.shape[-1] != 1:
            raise ValueError(f"depth must be [N, H, W, 1], got {tuple(depth.shape)}")
        return depth.detach().float().contiguous()


class GraphRegressorBase(RegressorBase):
    """A façade whose ``build`` is recorded as a layer graph and run by the native graph runtime
    (``MP_MODEL_GRAPH``, ``_graph.py``): the reference's helpers (conv_layer / max_pool / avg_pool
    / max_pool_4 / fc_layer, e.g. train_dense_hier_networks.py:2416-2455,
    train_hier_networks.py:535-579) record ops on symbolic tensors that carry the reference's
    attribute names.  Subclasses implement ``record(h, w, *head_sizes)`` and set ``_outputs``."""
    MODEL_KIND = _lib.MP_MODEL_GRAPH
    OUTPUT_ATTRS = ("output", "p_output", "r_output", "m_output", "i_output", "t_output")

    # ---- the reference's helpers, recording instead of building TF ops ----
    def conv_layer(self, bottom, in_channels, out_channels, name, filter_size=3, batchnorm=None,
                   stride=(1, 1, 1, 1)):
        if batchnorm is not None and name in batchnorm:
            raise NotImplementedError("conv_layer batchnorm= (batch-moment BN) is a training option")
        return self._g.conv(bottom, in_channels, out_channels, name, filter_size, stride[1])

    def max_pool(self, bottom, name):
        return self._g.pool(bottom, 2)

    def max_pool_4(self, bottom, name):
        return self._g.pool(bottom, 4)

    def avg_pool(self, bottom, name):
        return self._g.pool(bottom, 2, avg=True)

    def fc_layer(self, bottom, in_size, out_size, name):
        return self._g.fc(bottom, in_size, out_size, name)

    def _set(self, attr, t):
        t.label = attr
        setattr(self, attr, t)
        return t

    def _concat(self, attr, xs):
        return self._set(attr, self._g.concat(xs))

    def _relu_fc(self, attr_fc, attr_relu, x, in_size, out_size, name):
        f = self._set(attr_fc, self.fc_layer(x, in_size, out_size, name))
        return self._set(attr_relu, self._g.relu(f))   # dropout only when train_mode (never here)

    def _new_graph(self, h, w):
        from . import _graph
        self._g = _graph.GraphRecorder(int(h), int(w), 1)
        return self._g

    def _table(self, g) -> List[W.Var]:
        from . import _graph
        v: List[W.Var] = []
        for name, shp in _graph.layer_shapes(g).items():
            v += W._conv_b(name, shp[0], shp[2], shp[3]) if len(shp) == 4 else W._fc(f"cnn/{name}", *shp)
        return v

    def _on_context(self, ctx):
        from . import _graph
        _graph.install(ctx, self._g, self._outputs)

    def _graph_build(self, depth, heads, batch_norm, train_mode):
        depth = self._check_input(depth, batch_norm, train_mode)
        n, h, w, _ = depth.shape
        self.shapes = [int(s) for s in heads]
        key = (tuple(self.shapes), int(h), int(w))
        if getattr(self, "_rec_key", None) != key:
            self.record(h, w, *self.shapes)
            self._outputs = [getattr(self, a) for a in self.OUTPUT_ATTRS]
            self._rec_key = key
            self._ctx_key = None
        self._ctx = self._context(key, self._table(self._g), depth.device.index or 0)
        return self._graph_forward(depth)

    def _graph_forward(self, depth):
        import torch
        depth = depth.detach().float().contiguous()
        n = depth.shape[0]
        outs = [torch.empty((n, s), dtype=torch.float32, device=depth.device) for s in self.shapes]
        self._ctx.graph_fwd(depth, outs, _lib.current_stream(depth.device))
        for a, o in zip(self.OUTPUT_ATTRS, outs):
            setattr(self, a, o)
        return outs[0]
