"""Drop-in for the inference pieces of ``/root/reference/train_cnn_networks_hgru.py``: the attention
(centre-of-mass) regressor and the frame -> CoM -> crop -> pose chain of its ``test_model`` loop.

* ``attn_model_struct().build(images, num_dims)`` -> ``.out_put`` [N, num_dims]
  (train_cnn_networks_hgru.py:422-525): ``mp_attn_fwd`` -- TF1 bilinear resize to 128x128, five
  conv + max-pool + BN stages, afc_1 + relu + BN, afc_out, on the generic implicit-GEMM conv /
  split-K FC kernels (fp32 MFMA).
* ``prepare_data_test(images, tr_res, md, config)`` (61-74): with CUDA tensors it crops every
  frame on the GPU in one launch (``mp_crop3d_dev``), bit-exact with the host ``cropArea3D``
  integers, and the patches never leave the device; with numpy arrays it runs the native host
  crop (``mp_crop3d_batch``).
* ``FramePosePipeline``: ``test_model``'s per-batch body (284-321) -- attention, device crop,
  hGRU pose regressor -- as one device-resident call.
* ``cnn_model_struct().build(crops, num_classes)`` -> ``.out_put`` [N, num_classes]
  (train_cnn_networks_hgru.py:626-760): the regressor the reference's driver builds for
  validation (169), ``test_model`` (291) and ``eval_model_on_real_data`` (363) -- five conv +
  max-pool stages and four FCs, recorded op for op and run on the native layer-graph runtime.

Training (``train_model``: TFRecord queues, Adam, l2 losses) is outside the inference path.
``train_mode`` must be falsy: the reference's ``test_model`` builds the attention net with
``train_mode=True`` (dropout 0.7 and batch-statistics BN at test time, 287); that is a training
graph and raises here, as for the other facades.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import _lib
from . import weights as W
from ._regressor import GraphRegressorBase, RegressorBase


@dataclass
class InferenceConfig:
    """The ``config.py`` fields the inference chain reads (config.py:31-51)."""
    image_orig_size: List[int] = field(default_factory=lambda: [424, 512, 1])
    image_target_size: List[int] = field(default_factory=lambda: [128, 128, 1])
    image_max_depth: float = 10000.
    num_joints: int = 23
    num_dims: int = 3

    @property
    def num_classes(self) -> int:
        return self.num_joints * self.num_dims


class attn_model_struct(RegressorBase):
    """``attn_model_struct`` (train_cnn_networks_hgru.py:422-525), inference."""

    MODEL_KIND = _lib.MP_MODEL_ATTN

    def __init__(self, trainable=True):
        super().__init__(trainable)
        self._BATCH_NORM_DECAY = 0.997
        self._BATCH_NORM_EPSILON = 1e-5

    def build(self, depth, output_shape, batch_norm=None, train_mode=None):
        """``depth`` CUDA [N, H, W, 1] fp32 normalised frames (images / image_max_depth); any H, W
        (resized to 128 x 128).  Sets and returns ``.out_put`` [N, output_shape]."""
        depth = self._check_input(depth, batch_norm, train_mode)
        self.output_shape = int(output_shape)
        table = W.attn_vars(output_shape=self.output_shape)
        self._ctx = self._context(self.output_shape, table, depth.device.index or 0)
        return self.forward(depth)

    def forward(self, depth, out=None):
        import torch
        depth = depth.detach().float().contiguous()
        if out is None:
            out = torch.empty((depth.shape[0], self.output_shape), dtype=torch.float32, device=depth.device)
        self._ctx.attn_fwd(depth, out, _lib.current_stream(depth.device))
        self.out_put = out
        return out


class cnn_model_struct(GraphRegressorBase):
    """``cnn_model_struct`` (train_cnn_networks_hgru.py:626-760), inference: conv_1 .. conv_5 (3x3,
    conv_5 5x5; relu(conv2d SAME + b)) each with a 2x2 max pool, fc_1 .. fc_3 + relu, fc_4.  The
    reference's driver builds it for the validation / test crops (169, 291, 363).  ``build``
    records the reference's calls (``record``, op for op against the reference's AST in
    tests/test_cnn_model.py) and runs them on the layer-graph runtime (the f16x3 halo / tap-skipping
    convs fused with their max pools, split-K FCs)."""

    OUTPUT_ATTRS = ("out_put",)

    def record(self, h, w, output_shape):
        """The graph of build (639-673)."""
        g = self._new_graph(h, w)
        c, put = self.conv_layer, self._set
        prev = g.input                                                                       # 641
        for i, (name, k, cin, cout) in enumerate(W.CNN_CONV_SPECS, 1):                       # 642-656
            put(f"conv{i}", c(prev, cin, cout, name, filter_size=k))
            prev = put(f"pool{i}", self.max_pool(getattr(self, f"conv{i}"), f"pool_{i}"))
        flat = 1
        for s in self.pool5.shape:
            flat *= s
        r1 = self._relu_fc("fc1", "relu1", self.pool5, flat, 1024, "fc_1")                     # 658-661
        r2 = self._relu_fc("fc2", "relu2", r1, 1024, 1024, "fc_2")                            # 663-666
        r3 = self._relu_fc("fc3", "relu3", r2, 1024, 1024, "fc_3")                            # 668-671
        f4 = put("fc4", self.fc_layer(r3, 1024, int(output_shape), "fc_4"))                   # 672
        put("out_put", g.identity(f4))                                                        # 673
        return g

    def build(self, depth, output_shape, batch_norm=None, train_mode=None):
        """``depth`` CUDA [N, H, W, 1] fp32 crops (crop / 10000); sets and returns ``.out_put``
        [N, output_shape] (joint-major, / (cube_z / 2), as hgru_pose)."""
        return self._graph_build(depth, (output_shape,), batch_norm, train_mode)

    def forward(self, depth):
        return self._graph_forward(depth)


def prepare_data_test(image_np, tr_res, md, config, dsize: Optional[int] = None):
    """``prepare_data_test`` (train_cnn_networks_hgru.py:61-74): returns (patches [N, 128, 128, 1]
    = cropArea3D(image * max_depth, tr_res * [orig0, orig1, max_depth]) / max_depth, coms, Ms).

    CUDA tensors in -> everything stays on the device (``coms`` [N, 3] and ``Ms`` [N, 3, 3] float64
    tensors); numpy in -> the native host crop, ``coms`` / ``Ms`` as lists like the reference."""
    import torch
    dsize = int(dsize or config.image_target_size[0])
    scale = (float(config.image_orig_size[0]), float(config.image_orig_size[1]), float(config.image_max_depth))
    if isinstance(image_np, torch.Tensor) and image_np.is_cuda:
        patches, Ms, coms = md.crop_batch_device(image_np, tr_res, com_scale=scale,
                                                 frame_scale=float(config.image_max_depth), dsize=dsize)
        return patches, coms, Ms
    fr = np.asarray(image_np, np.float32)
    if fr.ndim == 4:
        fr = fr[..., 0]
    frames_mm = fr * np.float32(config.image_max_depth)
    coms_in = np.asarray(tr_res, np.float32).reshape(-1, 3) * np.array(scale)
    patches, Ms, coms = md.crop_batch(frames_mm, coms=coms_in, dsize=dsize)
    if float(md.maxDepth) != float(config.image_max_depth):
        raise ValueError("md.maxDepth must equal config.image_max_depth for the host batch crop")
    return patches, list(coms), [np.asmatrix(m) for m in Ms]


class FramePosePipeline:
    """``test_model``'s per-batch body (train_cnn_networks_hgru.py:284-321) on one GPU:
    frames -> attention CoM -> device crop -> hGRU pose, no host round trip in between.

    ``run(frames)`` returns (pose output [N, num_classes] normalised by cube_z / 2, coms [N, 3],
    Ms [N, 3, 3]); the caller maps to millimetres with ``md.getAbsoluteCoordinates`` as the
    reference does."""

    def __init__(self, attn: attn_model_struct, pose_model, md, config: Optional[InferenceConfig] = None,
                 check_crops: bool = True):
        self.attn, self.pose, self.md = attn, pose_model, md
        self.config = config or InferenceConfig()
        self.check_crops = check_crops

    def run(self, frames, h2_init=None):
        cfg = self.config
        com_norm = self.attn.build(frames, cfg.num_dims)
        patches, Ms, coms = self.md.crop_batch_device(
            frames, com_norm, com_scale=(cfg.image_orig_size[0], cfg.image_orig_size[1], cfg.image_max_depth),
            frame_scale=float(cfg.image_max_depth), dsize=cfg.image_target_size[0], check=self.check_crops)
        out = self.pose.build(patches, cfg.num_classes, h2_init=h2_init)
        return out, coms, Ms


class StreamPosePipeline:
    """SURVEY config 5, one depth frame per call: the host CoM crop of ``MonkeyDetector`` (native
    ``mp_crop3d_batch``) -> the hGRU pose forward at batch 1 -> absolute joints
    (``getAbsoluteCoordinates``, monkeydetector.py:356-360).  The reference's frame loop
    (train_cnn_networks_hgru.py:284-321 with the detector's ``cropArea3D`` in place of the attention
    net) minus the per-call allocations: the crop is written straight into a reused host buffer, one
    H2D and one D2H bracket the forward on the current stream.  ``pinned=True`` stages through pinned
    memory with asynchronous copies and waits on that stream alone; it measured no faster than the
    default pageable blocking copies at batch 1 (1.103 vs 1.097 ms p50, DESIGN.md §3a'').

    ``pose_model``: a built ``hgru_pose.model`` (weights loaded); ``h2_init``: an optional fixed
    [1, dsize / 2, dsize / 2, 64] CUDA hidden state (else the model's own hidden init).
    ``run(frame_mm)`` -> (joints_xyz [num_joints, 3] mm, joints_uvd [num_joints, 3], com_uvd [3])."""

    def __init__(self, pose_model, md, h2_init=None, dsize: int = 128, num_joints: int = 23, device=None,
                 pinned: bool = False):
        import torch
        self.pose, self.md, self.h2_init = pose_model, md, h2_init
        self.dsize, self.num_joints = int(dsize), int(num_joints)
        dev = torch.device(device) if device is not None else (
            h2_init.device if h2_init is not None else torch.device("cuda", torch.cuda.current_device()))
        self.pinned = bool(pinned)   # False: pageable staging, blocking copies (the copies' own waits)
        self._x_host = torch.empty((1, self.dsize, self.dsize, 1), dtype=torch.float32)
        if self.pinned:
            self._x_host = self._x_host.pin_memory()
        self._x_np = self._x_host.numpy()
        self._x_dev = torch.empty((1, self.dsize, self.dsize, 1), dtype=torch.float32, device=dev)
        self._y_host = torch.empty((1, self.num_joints * 3), dtype=torch.float32)
        if self.pinned:
            self._y_host = self._y_host.pin_memory()
        self._y_dev = torch.empty((1, self.num_joints * 3), dtype=torch.float32, device=dev)
        self._half_z = float(md.cube[2]) / 2.0
        self._dev = dev
        # with a given O0 the built context is called directly (no per-call façade work)
        self._direct = h2_init is not None and getattr(pose_model, "_ctx", None) is not None
        if self._direct:
            self._h2 = h2_init.detach().float().contiguous()

    def run(self, frame_mm, com=None, nthreads: int = 1):
        import torch
        ts = torch.cuda.current_stream(self._dev)   # the copies and the forward on the caller's stream
        _, _, coms = self.md.crop_batch(np.asarray(frame_mm, np.float32)[None], None if com is None else [com],
                                        dsize=self.dsize, nthreads=nthreads, out=self._x_np)
        self._x_dev.copy_(self._x_host, non_blocking=self.pinned)
        if self._direct:
            self.pose._ctx.pose_fwd(self._x_dev, self._h2, self._y_dev, ts.cuda_stream)
            out = self._y_dev
        else:
            out = self.pose.forward(self._x_dev, h2_init=self.h2_init)
        self._y_host.copy_(out, non_blocking=self.pinned)
        if self.pinned:
            ts.synchronize()
        rel = self._y_host.numpy().reshape(self.num_joints, 3) * np.float32(self._half_z)
        xyz, uvd = self.md.getAbsoluteCoordinates(rel, coms[0])
        return xyz, uvd, coms[0]
