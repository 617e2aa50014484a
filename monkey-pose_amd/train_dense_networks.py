"""Drop-in for the model class of ``/root/reference/train_dense_networks.py`` (inference).

``dense_model_struct().build(depth, output_shape)`` -> ``.output`` [N, output_shape]
(train_dense_networks.py:211-408).  The training / test drivers of that file (``train_model``,
``test_model``: TFRecord queues, Adam, pickled results) are outside the inference path.

Two engines, same numbers: by default ``build`` records the reference's graph-builder calls
(``record``, op for op against the reference's AST in tests/test_regressors.py) and runs them on
the native layer-graph runtime (its three scales run side by side on separate streams);
``use_graph=False`` runs the hand-written one-stream schedule behind ``mp_dense_fwd``.
"""
from __future__ import annotations

from . import _lib
from . import weights as W
from ._regressor import GraphRegressorBase


class dense_model_struct(GraphRegressorBase):
    """``dense_model_struct`` (train_dense_networks.py:211-509): 49 convs over three dense scales,
    avg-pooled FC towers, 1536 -> 1024 -> 512 -> output_shape."""

    OUTPUT_ATTRS = ("output",)

    def __init__(self, trainable=True, use_graph=True):
        super().__init__(trainable)
        self.use_graph = use_graph

    def record(self, h, w, output_shape):
        """The graph of build (223-408); layer widths W.DENSE_WIDTHS (250-373)."""
        g = self._new_graph(h, w)
        c, put, cat = self.conv_layer, self._set, self._concat
        s2 = [1, 2, 2, 1]
        put("conv0", c(g.input, 1, 12, "conv_0", filter_size=3))                                  # 226
        put("pool0", self.max_pool(self.conv0, "pool_0"))                                         # 227
        put("conv1_1", c(self.pool0, 12, 16, "conv_1_1", filter_size=3))                          # 230
        put("conv1_2", c(self.conv1_1, 16, 24, "conv_1_2", filter_size=3, stride=s2))
        put("conv1_3", c(self.conv1_2, 24, 32, "conv_1_3", filter_size=3, stride=s2))
        put("conv2_1", c(self.conv1_1, 16, 24, "conv_2_1", filter_size=3))                        # 236
        put("conv2_2_1", c(self.conv1_1, 16, 24, "conv_2_2_1", filter_size=3, stride=s2))
        put("conv2_2_2", c(self.conv1_2, 24, 32, "conv_2_2_2", filter_size=3))
        cat("conv2_2", [self.conv2_2_1, self.conv2_2_2])
        put("conv2_3_2", c(self.conv1_2, 24, 32, "conv_2_3_2", filter_size=3, stride=s2))
        put("conv2_3_3", c(self.conv1_3, 32, 48, "conv_2_3_3", filter_size=3))
        cat("conv2_3", [self.conv2_3_2, self.conv2_3_3])
        hist = {1: [self.conv1_1, self.conv2_1], 2: [self.conv1_2, self.conv2_2],
                3: [self.conv1_3, self.conv2_3]}
        for L in (3, 4, 5, 6):                                                                    # 248-373
            a, b, cc, d, e, f, gg, hh, i, j = W.DENSE_WIDTHS[L]
            q, n = f"conv{L}_", f"conv_{L}_"
            in1 = cat(q + "1_in", hist[1])
            put(q + "1_1x1", c(in1, in1.channels, a, n + "1_1x1", filter_size=1))
            o1 = put(q + "1", c(getattr(self, q + "1_1x1"), a, b, n + "1", filter_size=3))
            put(q + "2_1x1_1", c(in1, in1.channels, cc, n + "2_1x1_1", filter_size=1))
            o21 = put(q + "2_1", c(getattr(self, q + "2_1x1_1"), cc, d, n + "2_1", filter_size=3, stride=s2))
            in2 = cat(q + "2_in", hist[2])
            put(q + "2_1x1_2", c(in2, in2.channels, e, n + "2_1x1_2", filter_size=1))
            o22 = put(q + "2_2", c(getattr(self, q + "2_1x1_2"), e, f, n + "2_2", filter_size=3))
            o2 = cat(q + "2", [o21, o22])
            put(q + "3_1x1_2", c(in2, in2.channels, gg, n + "3_1x1_2", filter_size=1))
            o32 = put(q + "3_2", c(getattr(self, q + "3_1x1_2"), gg, hh, n + "3_2", filter_size=3, stride=s2))
            in3 = cat(q + "3_in", hist[3])
            put(q + "3_1x1_3", c(in3, in3.channels, i, n + "3_1x1_3", filter_size=1))
            o33 = put(q + "3_3", c(getattr(self, q + "3_1x1_3"), i, j, n + "3_3", filter_size=3))
            o3 = cat(q + "3", [o32, o33])
            for k, v in ((1, o1), (2, o2), (3, o3)):
                hist[k].append(v)
        pools = [put(f"pool{k}", self.avg_pool(getattr(self, f"conv6_{k}"), f"pool_{k}")) for k in (1, 2, 3)]   # 376-378
        relus = []
        for k, p in enumerate(pools, 1):                                                          # 381-396
            flat = 1
            for s in p.shape:
                flat *= s
            relus.append(self._relu_fc(f"fc1_{k}", f"relu1_{k}", p, flat, 512, f"fc_1_{k}"))
        cc3 = cat("concat", relus)                                                                # 398
        r2 = self._relu_fc("fc2", "relu2", cc3, 512 * 3, 1024, "fc_2")                           # 399-402
        r3 = self._relu_fc("fc3", "relu3", r2, 1024, 512, "fc_3")                                # 404-407
        f4 = put("fc4", self.fc_layer(r3, 512, int(output_shape), "fc_4"))                       # 408
        put("output", g.identity(f4))
        return g

    def build(self, depth, output_shape, batch_norm=None, train_mode=None):
        self.output_shape = int(output_shape)
        if self.use_graph:
            return self._graph_build(depth, (output_shape,), batch_norm, train_mode)
        depth = self._check_input(depth, batch_norm, train_mode)
        n, h, w, _ = depth.shape
        if h != w or h % 32:
            raise ValueError("dense_model_struct needs square crops with size % 32 == 0")
        table = W.dense_vars(output_shape=self.output_shape, crop=int(h))
        self._ctx = self._context((self.output_shape, int(h)), table, depth.device.index or 0,
                                  kind=_lib.MP_MODEL_DENSE)
        return self.forward(depth)

    def forward(self, depth):
        if self.use_graph:
            return self._graph_forward(depth)
        import torch
        depth = depth.detach().float().contiguous()
        out = torch.empty((depth.shape[0], self.output_shape), dtype=torch.float32, device=depth.device)
        self._ctx.dense_fwd(depth, out, _lib.current_stream(depth.device))
        self.output = out
        return out
