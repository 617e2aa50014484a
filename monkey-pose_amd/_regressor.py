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

    def load_weights(self, weights: Dict[str, np.ndarray]) -> None:
        self.weights = {(k if k.startswith("cnn/") else "cnn/" + k): v for k, v in weights.items()}
        self._ctx_key = None
        self._strict = False

    def load_checkpoint(self, path: str, remap=None, strict: bool = True) -> None:
        """Weights from a TF1 V2 checkpoint (see ``hgru_pose.model.load_checkpoint``)."""
        from . import tf_checkpoint as C
        t = C.model_variables(C.read_checkpoint(path))
        self.load_weights(remap(t) if remap else t)
        self._strict = strict

    def load_npz(self, path: str) -> None:
        with np.load(path, allow_pickle=False) as z:
            self.load_weights({k: z[k] for k in z.files})

    def _on_context(self, ctx: _lib.Context) -> None:
        """hook between mp_create and the weights (graph contexts install their graph here)"""

    def _table(self, **kw) -> List[W.Var]:
        raise NotImplementedError

    def _resolve(self, table) -> Dict[str, np.ndarray]:
        given = dict(self.weights or {})
        missing = [v.name for v in table if v.name not in given]
        if missing and getattr(self, "_strict", False) and self.data_dict is None:
            raise KeyError(f"checkpoint lacks {len(missing)} variable(s) the model needs: {missing[:8]}")
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
              'fp32': 'fp32', 'f32': 'fp32'}.get(self.compute_dtype)
        if dt is None:
            raise ValueError(f"regressor compute_dtype must be 'auto', 'fp32_split' or 'fp32', "
                             f"got {self.compute_dtype!r}")
        return dt

    def _context(self, key, table, device: int) -> _lib.Context:
        dt = self._dtype()
        key = (key, device, id(self.weights), id(self.data_dict), dt)
        if self._ctx is None or self._ctx_key != key:
            ctx = _lib.Context(self.MODEL_KIND, device)
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
