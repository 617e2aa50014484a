"""Drop-in for the model class of ``/root/reference/train_hier_networks.py`` (inference).

``hier_model_struct().build(depth, output_shape, P_shape, R_shape, M_shape, I_shape, T_shape)``
sets ``.output`` (whole hand, [N, output_shape]) and ``.p_output .. .t_output`` (per-limb heads)
(train_hier_networks.py:327-530).  Not a sequential cascade: ``output`` fuses the five limb
trunks; the limb heads are siblings.  The training / test drivers are outside the inference path.
"""
from __future__ import annotations

from . import _lib
from . import weights as W
from ._regressor import RegressorBase


class hier_model_struct(RegressorBase):
    MODEL_KIND = _lib.MP_MODEL_HIER

    def build(self, depth, output_shape, P_shape, R_shape, M_shape, I_shape, T_shape,
              batch_norm=None, train_mode=None):
        depth = self._check_input(depth, batch_norm, train_mode)
        n, h, w, _ = depth.shape
        if h != w or h % 64:
            raise ValueError("hier_model_struct needs square crops with size % 64 == 0")
        self.shapes = [int(output_shape), int(P_shape), int(R_shape), int(M_shape), int(I_shape),
                       int(T_shape)]
        table = W.hier_vars(output_shape=self.shapes[0], part_shapes=tuple(self.shapes[1:]),
                            crop=int(h))
        self._ctx = self._context((tuple(self.shapes), int(h)), table, depth.device.index or 0)
        return self.forward(depth)

    def forward(self, depth):
        import torch
        depth = depth.detach().float().contiguous()
        n = depth.shape[0]
        outs = [torch.empty((n, s), dtype=torch.float32, device=depth.device) for s in self.shapes]
        self._ctx.hier_fwd(depth, outs, _lib.current_stream(depth.device))
        (self.output, self.p_output, self.r_output, self.m_output, self.i_output,
         self.t_output) = outs
        return self.output
