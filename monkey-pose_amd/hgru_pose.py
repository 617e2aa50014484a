"""Drop-in for ``/root/reference/hgru_pose.py`` (inference): ``model().build(depth, output_shape)``.

Same class, attribute and argument names as the reference (``hgru_pose.py:6-118``).  ``build``
runs the forward immediately on the depth crops' device (the reference builds a TF graph that a
later ``sess.run`` executes) and sets ``self.out_put`` to a ``[N, output_shape]`` fp32 tensor in
the reference's joint-major layout (``j*3 + {x,y,z}``, normalised by ``cube_z / 2``).  Call
``forward(depth)`` to run again with the finalized weights.

Everything is computed by ``libmonkeypose.so`` (HIP, gfx950); there is no CPU path.
"""
from __future__ import annotations

import copy
from typing import Dict, Optional

import numpy as np

from . import _lib
from . import weights as W


class model:
    """``hgru_pose.model`` (hgru_pose.py:6-39)."""

    def __init__(self, trainable=True):
        self.trainable = trainable
        self.data_dict = None                  # {layer: [W, b]} as in get_var (hgru_pose.py:199)
        self.var_dict = {}
        self.SRF = 1
        self.SSN = 15
        self.SSF = 15
        self.strides = [1, 1, 1, 1]
        self._BATCH_NORM_DECAY = 0.997
        self._BATCH_NORM_EPSILON = 1e-5
        self.padding = 'SAME'
        self.timesteps = 8
        self.aux = {
            'recurrent_nl': 'tanh',
            'rectify_weights': None,
            'pre_batchnorm': False,
            'gate_filter': 1,
            'xi': False,
            'post_batchnorm': False,
            'dense_connections': False,
            'symmetric_weights': True,
            'symmetric_gate_weights': False,
            'batch_norm': False,
            'atrous_convolutions': False,
            'output_gru_gates': False,
            'association_field': True,
            'multiplicative_excitation': True,
            'gru_gates': True,
            'gamma': True,
            'adapation': True,
            'trainable': True,
        }
        self.weights: Optional[Dict[str, np.ndarray]] = None   # TF variable name -> array
        self.weight_seed = 1234
        # eCRF conv path (all fp32-class): 'auto' (default: FFT when the map allows, see
        # _lib.resolve_dtype), 'fp32_fft', 'fp32_split' (direct f16x3), 'fp32' (exact fp32 MFMA) or
        # 'bf16' (FFT path with bf16 spectral / gate GEMMs, ~1e-2 error; SURVEY config 4)
        self.compute_dtype = 'auto'
        self._ctx: Optional[_lib.Context] = None
        self._ctx_key = None
        self.out_put = None
        self.h2_init = None
        self._taps = None          # intermediates of the last forward (see _tap)
        self._last = None          # (depth, h2_init) of the last forward
        self.states_O = None       # build(..., store_states=True): [N, T, 64, 64, 64] per-step states
        self.states_I = None
        self.hidden_seed = 7       # hidden_init 'random' without h2_init: call c draws seed hidden_seed + c
        self._calls = 0
        self._rng_call = None
        self._ref_order = False

    def __getitem__(self, name):
        return getattr(self, name)

    def __contains__(self, name):
        return hasattr(self, name)

    # ---------------------------------------------------------------- weights
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
        """Weights from a TF1 V2 checkpoint (prefix, ``.index`` path or directory; see
        ``tf_checkpoint``), optimizer slots dropped; ``remap`` maps the name dict first (e.g. the
        pose half of ``tf_checkpoint.split_hgru_train_checkpoint``).  ``strict``: build() raises
        if a variable the model needs is absent instead of synthesising it."""
        from . import tf_checkpoint as C
        t = C.model_variables(C.read_checkpoint(path))
        self.load_weights(remap(t) if remap else t, synthesize_missing=not strict)

    def load_npz(self, path: str, synthesize_missing: bool = False) -> None:
        with np.load(path, allow_pickle=False) as z:
            self.load_weights({k: z[k] for k in z.files}, synthesize_missing)

    def _resolve_weights(self, output_shape: int, crop=(128, 128)) -> Dict[str, np.ndarray]:
        table = W.hgru_pose_vars(output_shape=output_shape, timesteps=self.timesteps, crop=crop)
        given = dict(self.weights or {})
        out: Dict[str, np.ndarray] = {}
        covered = set()
        for layer in (self.data_dict or {}):
            covered |= {f"cnn/{layer}/{layer}{s}" for s in ("_weights", "_biases", "_filters")}
        missing = [v.name for v in table if v.name not in given and v.name not in covered]
        if missing and self.weights is not None and getattr(self, "_strict", True):
            raise KeyError(f"the loaded weights lack {len(missing)} variable(s) the model needs "
                           f"(load_weights(..., synthesize_missing=True) fills them): {missing[:8]}")
        for v in table:
            if v.name in given:
                out[v.name] = np.asarray(given[v.name], np.float32)
            else:
                out[v.name] = W.synth_value(v, self.weight_seed, self.timesteps)
        # data_dict[name] = [W, b] overrides conv_* / fc_* (get_var, hgru_pose.py:199-200)
        if self.data_dict is not None:
            for layer, vals in self.data_dict.items():
                suff = ("_weights", "_biases") if layer.startswith("fc") else ("_filters", "_biases")
                for idx in (0, 1):
                    out[f"cnn/{layer}/{layer}{suff[idx]}"] = np.asarray(vals[idx], np.float32)
        for k, v in out.items():
            self.var_dict[(k.split("/")[1], k)] = v
        return out

    def _context(self, output_shape: int, device: int, crop=(128, 128)) -> _lib.Context:
        dtype = _lib.resolve_dtype(self.compute_dtype, crop[0] // 2, crop[1] // 2)
        key = (output_shape, device, tuple(crop), id(self.weights), id(self.data_dict), dtype)
        if self._ctx is None or self._ctx_key != key:
            ctx = _lib.Context(_lib.MP_MODEL_HGRU_POSE, device)
            for name, val in self._resolve_weights(output_shape, crop).items():
                ctx.set_weight(name, val)
            ctx.finalize(_lib.dtype_code(dtype))
            self._ctx, self._ctx_key = ctx, key
        return self._ctx

    # ---------------------------------------------------------------- forward
    # ------------------------------------------------------- reference intermediates (hgru_pose.py:50-103)
    def _tap(self, name):
        """The reference's graph tensors m.conv1 ... m.relu1.  In TF they are evaluated on demand;
        here the first access re-runs the last forward once with every tap requested
        (mp_hgru_pose_fwd_taps; the forward is deterministic, so out_put is unchanged), unless
        build(..., keep_intermediates=True) already captured them."""
        if self._taps is None:
            if self._last is None:
                raise AttributeError(f"{name}: call build() first")
            self._run(*self._last, keep=True)
        return self._taps[name]

    conv1 = property(lambda self: self._tap("conv1"))
    pool1 = property(lambda self: self._tap("pool1"))
    conv2 = property(lambda self: self._tap("conv2"))
    conv3 = property(lambda self: self._tap("conv3"))
    hgru = property(lambda self: self._tap("hgru"))
    fc1 = property(lambda self: self._tap("fc1"))
    relu1 = property(lambda self: self._tap("relu1"))

    def build(self, depth, output_shape, batch_norm=None, train_mode=None, h2_init=None,
              keep_intermediates=False, dtype=None, store_states=False, reference_stack_order=False):
        """``hgru_pose.model.build`` (hgru_pose.py:47-105), inference only.

        depth     torch CUDA tensor [N, 128, 128, 1] fp32 (crop / 10000, train_cnn_networks_hgru.py:50)
        h2_init   optional [N, 64, 64, 64] initial hGRU output state for ``aux['hidden_init'] ==
                  'random'`` (the default).  Without it the state is drawn on the device for every
                  call, as the reference redraws it per run (hgru_module.py:879-887): call c of
                  this model draws ``weights.synth_hidden((N, 64, 64, 64), seed=self.hidden_seed
                  + c)`` bit for bit, no host RNG and no copy.  'zeros' / 'identity' (888-890,
                  876-878) need none.
        dtype     None (keep ``compute_dtype``), 'fp32' (fp32-class, fastest path for the map:
                  ``compute_dtype = 'auto'``) or 'bf16' (bf16 spectral / gate GEMMs on the FFT path)
        store_states  also keep every hGRU timestep's states (the circuit's ``store_states``,
                  hgru_module.py:889-915) as ``self.states_O`` / ``self.states_I``, each
                  [N, T, 64, 64, 64]: O_t after the rho gain and I_t.  (With
                  ``aux['store_states']`` the reference itself would feed the 5-D stack into fc_1;
                  that configuration is rejected.)  ``reference_stack_order=True`` gives the
                  reference's own interleaved stacks instead (``hgru_module.reference_stacks``).
        """
        if dtype is not None:
            if dtype not in ('fp32', 'bf16'):
                raise ValueError("dtype must be 'fp32' or 'bf16'")
            self.compute_dtype = 'auto' if dtype == 'fp32' else 'bf16'
        import torch
        if train_mode:
            raise NotImplementedError("train_mode=True (dropout / BN batch statistics / backward) is "
                                      "outside the inference path")
        if batch_norm is not None:
            raise NotImplementedError("conv_layer batchnorm= option is never used by hgru_pose")
        if not isinstance(depth, torch.Tensor) or not depth.is_cuda:
            raise TypeError("depth must be a CUDA (ROCm) torch tensor")
        if depth.dim() != 4 or depth.shape[-1] != 1:
            raise ValueError(f"depth must be [N, H, W, 1], got {tuple(depth.shape)}")
        self.output_shape = int(output_shape)
        self._hidden_init()   # validate the aux before any work
        self._ctx = self._context(self.output_shape, depth.device.index or 0,
                                  (int(depth.shape[1]), int(depth.shape[2])))
        self._ref_order = bool(reference_stack_order)
        return self.forward(depth, h2_init, keep_intermediates, store_states)

    def _hidden_init(self) -> str:
        hi = self.aux.get('hidden_init', 'random')
        if hi not in _lib.MP_HIDDEN:
            raise NotImplementedError(f"aux hidden_init={hi!r}: the reference raises (hgru_module.py:891-892)")
        if self.aux.get('store_states', False):
            raise NotImplementedError("aux store_states=True makes hgru_layer return the [N, T, ...] stack, "
                                      "which fc_1 cannot take; use build(..., store_states=True)")
        return hi

    def forward(self, depth, h2_init=None, keep_intermediates=False, store_states=False):
        import torch
        if self._ctx is None:
            raise RuntimeError("call build() first")
        depth = depth.detach().float().contiguous()
        n, h, w, _ = depth.shape
        hi = self._hidden_init()
        self._rng_call = None
        if hi == 'random':
            if h2_init is None:
                self._rng_call = self._calls     # MP_HIDDEN_RANDOM: the library draws O0
                self._calls += 1
            else:
                h2_init = h2_init.detach().float().contiguous()
                if tuple(h2_init.shape) != (n, h // 2, w // 2, 64):
                    raise ValueError(f"h2_init must be [{n}, {h // 2}, {w // 2}, 64]")
        elif h2_init is not None:
            raise ValueError(f"h2_init is only used with aux hidden_init='random' (got {hi!r})")
        self.h2_init = h2_init
        self._last = (depth, h2_init)
        self._taps = None
        self.states_O = self.states_I = None
        return self._run(depth, h2_init, keep_intermediates, store_states)

    @property
    def last_hidden_call(self):
        """The call index whose device draw of O0 the last forward used (None when it was given
        ``h2_init`` or its aux hidden_init is not 'random')."""
        return self._rng_call

    def hidden_draw(self, call=None, batch=None, crop=(128, 128)):
        """The O0 that call ``call`` (default: the last forward's, ``last_hidden_call``) of this model
        drew on the device, recomputed on the host bit for bit: ``weights.synth_hidden((N, h/2, w/2,
        64), seed=hidden_seed + call)`` as a float32 numpy array.  Passing it back as ``h2_init``
        reproduces that call's output exactly."""
        if call is None:
            call = self._rng_call
            if call is None:
                raise ValueError("the last forward did not draw O0 on the device")
        if batch is None:
            if self._last is None:
                raise ValueError("give batch= (no forward has run yet)")
            batch, crop = self._last[0].shape[0], tuple(self._last[0].shape[1:3])
        return W.synth_hidden((batch, crop[0] // 2, crop[1] // 2, 64), seed=self.hidden_seed + call)

    def _run(self, depth, h2_init, keep=False, store_states=False):
        import torch
        n, h, w, _ = depth.shape
        dev = depth.device
        out = torch.empty((n, self.output_shape), dtype=torch.float32, device=dev)
        stream = _lib.current_stream(dev)
        hidden = _lib.MP_HIDDEN[self._hidden_init()]
        call = getattr(self, "_rng_call", None)
        if hidden == _lib.MP_HIDDEN_GIVEN and h2_init is None and call is not None:
            hidden = _lib.MP_HIDDEN_RANDOM      # re-running a tap replays the same call's draw
        hh, ww = h // 2, w // 2
        taps = {}
        if keep:
            shapes = {"conv1": (n, h, w, 64), "pool1": (n, hh, ww, 64), "conv2": (n, hh, ww, 64),
                      "conv3": (n, hh, ww, 64), "hgru": (n, hh, ww, 64), "fc1": (n, 1024), "relu1": (n, 1024)}
            taps = {k: torch.empty(v, dtype=torch.float32, device=dev) for k, v in shapes.items()}
        if store_states:
            T = self._ctx.info("timesteps")
            for k in _lib.STATE_NAMES:
                taps[k] = torch.empty((n, T, hh, ww, 64), dtype=torch.float32, device=dev)
        if taps or hidden:
            self._ctx.pose_fwd_taps(depth, h2_init, out, taps, stream, hidden, self.hidden_seed, call or 0)
        else:
            self._ctx.pose_fwd(depth, h2_init, out, stream)
        if keep:
            self._taps = {k: taps[k] for k in _lib.TAP_NAMES}
        if store_states:
            self.states_O, self.states_I = taps["states_O"], taps["states_I"]
            if self._ref_order:
                from .hgru_module import reference_stacks
                self.states_O, self.states_I = reference_stacks(self.states_O, self.states_I)
        self.out_put = out
        return out

    # ---------------------------------------------------------------- profiling
    def profile(self, enable: bool = True) -> None:
        self._ctx.profile(enable)

    def profile_read(self, name: str):
        return self._ctx.profile_read(name)
