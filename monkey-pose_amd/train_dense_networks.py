"""Drop-in for the model class of ``/root/reference/train_dense_networks.py`` (inference).

``dense_model_struct().build(depth, output_shape)`` -> ``.output`` [N, output_shape]
(train_dense_networks.py:211-408).  The training / test drivers of that file (``train_model``,
``test_model``: TFRecord queues, Adam, pickled results) are outside the inference path.
"""
from __future__ import annotations

from . import _lib
from . import weights as W
from ._regressor import RegressorBase


class dense_model_struct(RegressorBase):
    """``dense_model_struct`` (train_dense_networks.py:211-509): 49 convs over three dense scales,
    avg-pooled FC towers, 1536 -> 1024 -> 512 -> output_shape."""

    MODEL_KIND = _lib.MP_MODEL_DENSE

    def build(self, depth, output_shape, batch_norm=None, train_mode=None):
        import torch
        depth = self._check_input(depth, batch_norm, train_mode)
        n, h, w, _ = depth.shape
        if h != w or h % 32:
            raise ValueError("dense_model_struct needs square crops with size % 32 == 0")
        self.output_shape = int(output_shape)
        table = W.dense_vars(output_shape=self.output_shape, crop=int(h))
        self._ctx = self._context((self.output_shape, int(h)), table, depth.device.index or 0)
        return self.forward(depth)

    def forward(self, depth):
        import torch
        depth = depth.detach().float().contiguous()
        out = torch.empty((depth.shape[0], self.output_shape), dtype=torch.float32, device=depth.device)
        self._ctx.dense_fwd(depth, out, _lib.current_stream(depth.device))
        self.output = out
        return out
