"""Drop-in for the model class of ``/root/reference/train_hier_networks.py`` (inference).

``hier_model_struct().build(depth, output_shape, P_shape, R_shape, M_shape, I_shape, T_shape)``
sets ``.output`` (whole hand, [N, output_shape]) and ``.p_output .. .t_output`` (per-limb heads)
(train_hier_networks.py:327-530).  Not a sequential cascade: ``output`` fuses the five limb
trunks; the limb heads are siblings.  The training / test drivers are outside the inference path.

Two engines, same numbers: by default ``build`` records the reference's graph-builder calls
(``record``, op for op against the reference's AST in tests/test_regressors.py) and runs them on
the native layer-graph runtime (``MP_MODEL_GRAPH``), whose multi-stream schedule runs the three
trunks and five limb branches side by side; ``use_graph=False`` runs the hand-written one-stream
schedule behind ``mp_hier_fwd`` (``MP_MODEL_HIER``, the C-ABI entry point).
"""
from __future__ import annotations

from . import _lib
from . import weights as W
from ._regressor import GraphRegressorBase

FINGERS = ("p", "r", "m", "i", "t")


class hier_model_struct(GraphRegressorBase):
    def __init__(self, trainable=True, use_graph=True):
        super().__init__(trainable)
        self.use_graph = use_graph

    # ---- recorded graph of build (338-530) ----
    def _limb(self, f, src, size):
        """limb f (354-372): con_5 3x3 -> pool -> con_6 5x5 -> pool -> fc_1 -> fc_2 -> fc_3."""
        c5 = self._set(f"{f}_conv5", self.conv_layer(src, 512, 512, f"{f}_con_5", filter_size=3))
        p5 = self._set(f"{f}_pool5", self.max_pool(c5, f"{f}_pool_5"))
        c6 = self._set(f"{f}_conv6", self.conv_layer(p5, 512, 1024, f"{f}_con_6", filter_size=5))
        p6 = self._set(f"{f}_pool6", self.max_pool(c6, f"{f}_pool_6"))
        flat = 1
        for s in p6.shape:
            flat *= s
        r1 = self._relu_fc(f"{f}_fc1", f"{f}_relu1", p6, flat, 1024, f"{f}_fc_1")
        r2 = self._relu_fc(f"{f}_fc2", f"{f}_relu2", r1, 1024, 1024, f"{f}_fc_2")
        f3 = self._set(f"{f}_fc3", self.fc_layer(r2, 1024, size, f"{f}_fc_3"))
        self._set(f"{f}_output", self._g.identity(f3))
        return p6, flat

    def _trunk(self, br, src):
        """trunk br (347-352): con_3 128->256 -> pool -> con_4 256->512 -> pool."""
        c3 = self._set(f"{br}_conv3", self.conv_layer(src, 128, 256, f"{br}_con_3", filter_size=3))
        p3 = self._set(f"{br}_pool3", self.max_pool(c3, f"{br}_pool_3"))
        c4 = self._set(f"{br}_conv4", self.conv_layer(p3, 256, 512, f"{br}_con_4", filter_size=3))
        return self._set(f"{br}_pool4", self.max_pool(c4, f"{br}_pool_4"))

    def record(self, h, w, output_shape, P_shape, R_shape, M_shape, I_shape, T_shape):
        g = self._new_graph(h, w)
        sizes = dict(zip(FINGERS, (P_shape, R_shape, M_shape, I_shape, T_shape)))
        c1 = self._set("conv1", self.conv_layer(g.input, 1, 64, "conv_1", filter_size=3))        # 341
        p1 = self._set("pool1", self.max_pool(c1, "pool_1"))
        c2 = self._set("conv2", self.conv_layer(p1, 64, 128, "conv_2", filter_size=3))           # 344
        p2 = self._set("pool2", self.max_pool(c2, "pool_2"))
        pools = {}
        pr = self._trunk("pr", p2)                                                                # 347-352
        pools["p"] = self._limb("p", pr, int(sizes["p"]))                                         # 354-372
        pools["r"] = self._limb("r", pr, int(sizes["r"]))                                         # 374-393
        mi = self._trunk("mi", p2)                                                                # 395-400
        pools["m"] = self._limb("m", mi, int(sizes["m"]))                                         # 402-421
        pools["i"] = self._limb("i", mi, int(sizes["i"]))                                         # 423-442
        # limb T (444-469): its own con_3 / con_4 feed its con_5 directly
        c3 = self._set("t_conv3", self.conv_layer(p2, 128, 256, "t_con_3", filter_size=3))
        t3 = self._set("t_pool3", self.max_pool(c3, "t_pool_3"))
        c4 = self._set("t_conv4", self.conv_layer(t3, 256, 512, "t_con_4", filter_size=3))
        t4 = self._set("t_pool4", self.max_pool(c4, "t_pool_4"))
        pools["t"] = self._limb("t", t4, int(sizes["t"]))
        hand = []
        for f in FINGERS:                                                                         # 471-523
            p6, flat = pools[f]
            r1 = self._relu_fc(f"{f}h_fc1", f"{f}h_relu1", p6, flat, 1024, f"{f}h_fc_1")
            hand.append(self._relu_fc(f"{f}h_fc2", f"{f}h_relu2", r1, 1024, 1024, f"{f}h_fc_2"))
        hc = self._concat("h_concat", hand)                                                       # 525
        fr = self._relu_fc("final_fc1", "final_relu1", hc, 1024 * 5, 1024, "final_fc_1")         # 526-528
        f2 = self._set("final_fc2", self.fc_layer(fr, 1024, int(output_shape), "final_fc_2"))    # 529
        self._set("output", g.identity(f2))                                                       # 530
        return g

    # ---- build / forward ----
    def build(self, depth, output_shape, P_shape, R_shape, M_shape, I_shape, T_shape,
              batch_norm=None, train_mode=None):
        heads = (output_shape, P_shape, R_shape, M_shape, I_shape, T_shape)
        if self.use_graph:
            return self._graph_build(depth, heads, batch_norm, train_mode)
        depth = self._check_input(depth, batch_norm, train_mode)
        n, h, w, _ = depth.shape
        if h != w or h % 64:
            raise ValueError("hier_model_struct needs square crops with size % 64 == 0")
        self.shapes = [int(s) for s in heads]
        table = W.hier_vars(output_shape=self.shapes[0], part_shapes=tuple(self.shapes[1:]),
                            crop=int(h))
        self._ctx = self._context((tuple(self.shapes), int(h)), table, depth.device.index or 0,
                                  kind=_lib.MP_MODEL_HIER)
        return self.forward(depth)

    def forward(self, depth):
        if self.use_graph:
            return self._graph_forward(depth)
        import torch
        depth = depth.detach().float().contiguous()
        n = depth.shape[0]
        outs = [torch.empty((n, s), dtype=torch.float32, device=depth.device) for s in self.shapes]
        self._ctx.hier_fwd(depth, outs, _lib.current_stream(depth.device))
        for a, o in zip(self.OUTPUT_ATTRS, outs):
            setattr(self, a, o)
        return outs[0]
