"""Drop-in for ``/root/reference/hgru_module.py``: ``ContextualCircuit(X, ...).build()``.

Supports the configuration the pose model uses (``hgru_pose.py:20-39`` merged over the defaults
of ``auxilliary_variables``, ``hgru_module.py:9-51``): association-field eCRF with a full
SSFxSSF conv, 1x1 GRU gates on the input, multiplicative excitation, learned gamma/kappa/omega,
adaptation (rho), xi = zeta = 1, tanh recurrence, no rectification, with any ``hidden_init``
('random', 'zeros', 'identity') and ``store_states``.  Other aux combinations raise
``NotImplementedError`` rather than silently computing something else.  Inference only.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np

from . import _lib
from . import weights as W

# the effective aux of hgru_pose (hgru_pose.py:20-39 over hgru_module.py:9-51)
SUPPORTED_AUX = {
    'recurrent_nl': 'tanh', 'rectify_weights': None, 'gate_filter': 1, 'xi': False,
    'zeta': False, 'gamma': True, 'beta': True, 'nu': True, 'batch_norm': False,
    'atrous_convolutions': False, 'output_gru_gates': False, 'association_field': True,
    'multiplicative_excitation': True, 'gru_gates': True, 'adapation': True,
    'dense_connections': False, 'integration_type': 'alternate',
    'lesion_beta': False, 'lesion_nu': False, 'lesion_omega': False, 'lesion_kappa': False,
    'dropout': None,
}
# keys with more than one implemented value (build(), hgru_module.py:872-959)
CHOICE_AUX = {'hidden_init': ('random', 'zeros', 'identity'), 'store_states': (False, True)}
# keys that only affect training / initialisation, never the forward values
_IGNORED = {'symmetric_weights', 'symmetric_gate_weights', 'trainable', 'pre_batchnorm',
            'post_batchnorm', 'train', 'normal_initializer', 'gate_bias_init', 'dtype',
            'return_weights', 'lesions', 'tuning_nl', 'gate_nl', 'ecrf_nl', 'post_tuning_nl'}

_DEFAULTS = {  # auxilliary_variables() values for the keys checked above (hgru_module.py:13-51)
    'recurrent_nl': 'tanh', 'rectify_weights': None, 'gate_filter': 1, 'xi': False, 'zeta': False,
    'gamma': True, 'beta': True, 'nu': True, 'batch_norm': False, 'atrous_convolutions': False,
    'output_gru_gates': False, 'association_field': True, 'multiplicative_excitation': True,
    'gru_gates': False, 'adapation': False, 'dense_connections': False,
    'integration_type': 'alternate', 'hidden_init': 'random', 'lesion_beta': False,
    'lesion_nu': False, 'lesion_omega': False, 'lesion_kappa': False, 'dropout': None,
    'store_states': False,
}


class ContextualCircuit(object):
    """``hgru_module.ContextualCircuit`` (hgru_module.py:54-128)."""

    def __getitem__(self, name):
        return getattr(self, name)

    def __contains__(self, name):
        return hasattr(self, name)

    def __init__(self, X, timesteps=1, SRF=1, SSN=9, SSF=29, strides=[1, 1, 1, 1],
                 padding='SAME', aux=None, train=True):
        self.X = X
        self.n, self.h, self.w, self.k = [int(x) for x in X.shape]
        self.timesteps = timesteps
        self.strides = strides
        self.padding = padding
        self.train = train
        merged = dict(_DEFAULTS)
        if aux is not None and isinstance(aux, dict):
            for key, val in aux.items():
                merged[key] = val
        if merged.get('recurrent_nl') is not None and not isinstance(merged['recurrent_nl'], str):
            raise NotImplementedError("recurrent_nl must be given by name ('tanh')")
        bad = {k: merged[k] for k in SUPPORTED_AUX if merged.get(k) != SUPPORTED_AUX[k]}
        if bad:
            raise NotImplementedError(f"aux settings outside the implemented hGRU variant: {bad}")
        bad = {k: merged[k] for k, ok in CHOICE_AUX.items() if merged.get(k) not in ok}
        if bad:
            raise NotImplementedError(f"aux values outside {CHOICE_AUX}: {bad}")
        unknown = set(merged) - set(SUPPORTED_AUX) - set(CHOICE_AUX) - _IGNORED
        if unknown:
            raise NotImplementedError(f"unsupported aux keys: {sorted(unknown)}")
        for key, val in merged.items():
            setattr(self, key, val)
        self.SRF, self.SSN, self.SSF = SRF, SSN, SSF
        if isinstance(SSF, list):
            raise NotImplementedError("hierarchical (list) SSF is not implemented")
        self.SSF_ext = 2 * int(math.floor(SSF / 2.0)) + 1                # hgru_module.py:97
        if list(strides) != [1, 1, 1, 1] or padding != 'SAME':
            raise NotImplementedError("only strides [1,1,1,1] with SAME padding")
        self.p_shape = [self.SSF_ext, self.SSF_ext, self.k, self.k]
        self.i_shape = [self.gate_filter, self.gate_filter, self.k, self.k]
        self.o_shape = [self.gate_filter, self.gate_filter, self.k, self.k]
        self.bias_shape = [1, 1, 1, self.k]
        self.weights: Optional[Dict[str, np.ndarray]] = None
        self.weight_seed = 1234
        self.hidden_seed = 7        # hidden_init 'random': call c draws synth_hidden(seed=hidden_seed + c)
        self._calls = 0
        self.scope = "contextual_circuit"

    def prepare_tensors(self, weights: Optional[Dict[str, np.ndarray]] = None,
                        seed: Optional[int] = None) -> Dict[str, np.ndarray]:
        """Variables of ``prepare_tensors`` (hgru_module.py:172-503) keyed
        ``contextual_circuit/<name>``; given values win, the rest are synthesised."""
        table = W.hgru_circuit_vars(k=self.k, ssf=self.SSF_ext, gate_filter=self.gate_filter,
                                    timesteps=self.timesteps, scope=self.scope)
        given = {}
        for k_, v in (weights or self.weights or {}).items():
            given[k_.split("/")[-1]] = v
        s = self.weight_seed if seed is None else seed
        out = {}
        for v in table:
            short = v.name.split("/")[-1]
            out[v.name] = (np.asarray(given[short], np.float32) if short in given
                           else W.synth_value(v, s, self.timesteps))
        return out

    def build(self, weights: Optional[Dict[str, np.ndarray]] = None, h2_init=None,
              compute_dtype: str = 'auto', reference_stack_order: bool = False):
        """Run the circuit; returns ``(O, weights, activities)`` like the reference with
        ``return_weights=True`` (hgru_module.py:939-954).  ``compute_dtype``: 'auto' (the FFT
        path when the map allows), 'fp32_fft', 'fp32_split', 'fp32' or 'bf16' (see
        include/monkeypose.h and _lib.resolve_dtype).

        hidden_init (875-892): 'random' -> O0 = ``h2_init`` if given, else a fresh xavier-uniform
        draw made on the device for every call, as the reference redraws it every sess.run (the
        draw of call c is ``weights.synth_hidden(shape, seed=self.hidden_seed + c)``, bit for bit);
        'zeros' -> zeros_like(X), 'identity' -> X.
        store_states (889-915): O is the per-step stack ``[n, T, h, w, k]`` (O_t after the rho
        gain, 909-912) and ``weights['store_O']`` / ``weights['store_I']`` hold the O_t / I_t
        stacks.  (The reference's TensorArrays trade places every step -- ``full`` takes
        ``(store_O, store_I)`` where the loop passes ``(store_I, store_O)``, 825 vs 897-908 -- so
        its stacked "O" alternates O_t and I_t; here each stack holds what its name says.
        ``reference_stack_order=True`` returns the reference's interleaved stacks instead, see
        ``reference_stacks``.)"""
        import torch
        X = self.X
        if not isinstance(X, torch.Tensor) or not X.is_cuda:
            raise TypeError("X must be a CUDA (ROCm) torch tensor [n, h, w, k]")
        wts = self.prepare_tensors(weights)
        ctx = _lib.Context(_lib.MP_MODEL_HGRU_CIRCUIT, X.device.index or 0)
        for name, val in wts.items():
            ctx.set_weight(name, val)
        ctx.finalize(_lib.dtype_code(_lib.resolve_dtype(compute_dtype, X.shape[1], X.shape[2])))
        X = X.detach().float().contiguous()
        hidden = _lib.MP_HIDDEN[self.hidden_init]
        call = 0
        if self.hidden_init == 'random':
            if h2_init is None:
                hidden = _lib.MP_HIDDEN_RANDOM          # drawn on the device, per call
                call = self._calls
                self._calls += 1
            else:
                h2_init = h2_init.detach().float().contiguous()
                if h2_init.shape != X.shape:
                    raise ValueError("h2_init must have the shape of X")
        elif h2_init is not None:
            raise ValueError(f"h2_init is only used with hidden_init='random' (got {self.hidden_init!r})")
        O = torch.empty_like(X)
        sO = sI = None
        if self.store_states:
            sO = torch.empty((X.shape[0], self.timesteps) + tuple(X.shape[1:]), dtype=torch.float32,
                             device=X.device)
            sI = torch.empty_like(sO)
        ctx.circuit_fwd(X, h2_init, O, self.timesteps, _lib.current_stream(X.device), hidden, sO, sI,
                        rng_seed=self.hidden_seed, rng_call=call)
        torch.cuda.current_stream(X.device).synchronize()
        ctx.close()
        self.h2_init = h2_init
        weights_out = {k_.split("/")[-1]: v for k_, v in wts.items()}
        weights_out['p_t'] = weights_out['p_r']
        if self.store_states:
            if reference_stack_order:
                sO, sI = reference_stacks(sO, sI)
            weights_out['store_O'], weights_out['store_I'] = sO, sI
            return sO, weights_out, {}
        return O, weights_out, {}


def reference_stacks(states_O, states_I):
    """The reference's own ``store_states`` stacks from the per-step O_t / I_t stacks [n, T, ...].

    ``full(self, i0, O, I, store_O=None, store_I=None)`` (hgru_module.py:825) is called by
    ``tf.while_loop`` with the loop variables ``[i0, O, I, store_I, store_O]`` (897-908) and returns
    them in its own parameter order (857), so the two TensorArrays trade places every step: after
    T steps the array returned as ``store_O`` (912-914) holds O_t where T-1-t is even and I_t
    elsewhere, and ``store_I`` the complement (pinned symbolically, tests/test_hgru_structure.py).
    Returns (O_ref, I_ref) with the reference's layout, for callers that relied on it."""
    import torch
    T = states_O.shape[1]
    pick = torch.tensor([(T - 1 - t) % 2 == 0 for t in range(T)], device=states_O.device)
    pick = pick.view((1, T) + (1,) * (states_O.dim() - 2))
    return torch.where(pick, states_O, states_I), torch.where(pick, states_I, states_O)
