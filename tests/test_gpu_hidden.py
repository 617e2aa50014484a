"""hidden_init 'random' drawn on the device per call (hgru_module.py:879-887; MP_HIDDEN_RANDOM).

Without ``h2_init`` every call of a model draws a fresh O0 on the GPU, as the reference re-draws it
per ``sess.run``.  The draw of call c is ``weights.synth_hidden(shape, seed=hidden_seed + c)`` bit
for bit, so each call equals the explicit-``h2_init`` call with that host draw, bit for bit."""
import numpy as np
import pytest

from helpers import HGRU_POSE_AUX, MG, golden_meta, pkg

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).cuda()


@pytest.mark.parametrize("dtype", ["fp32_fft", "bf16"])
def test_pose_default_hidden_is_a_fresh_device_draw(dtype):
    mp = pkg()
    W = mp.weights
    meta = golden_meta()["pose_c128_t8"]
    n = 3
    wts, depth, _ = MG.pose_inputs(n, 128, 8, meta["weight_seed"], meta["crop_seed"], meta["o0_seed"])
    m = mp.hgru_pose.model()
    m.compute_dtype = 'auto' if dtype == 'fp32_fft' else dtype
    m.load_weights(wts)
    x = _cuda(depth)
    a = m.build(x, 69).cpu().numpy()                         # call 0: device draw, seed 7
    b = m.forward(x).cpu().numpy()                           # call 1: seed 8
    assert not np.array_equal(a, b)                          # re-drawn per call
    ref = mp.hgru_pose.model()
    ref.compute_dtype = m.compute_dtype
    ref.load_weights(wts)
    for c, got in ((0, a), (1, b)):
        o0 = W.synth_hidden((n, 64, 64, 64), seed=m.hidden_seed + c)
        exp = ref.build(x, 69, h2_init=_cuda(o0)).cpu().numpy()
        assert np.array_equal(got, exp), c
    # a tap read after the call replays that call's draw: out_put is unchanged
    m.forward(x)
    out = m.out_put.cpu().numpy()
    _ = m.conv3
    assert np.array_equal(m.out_put.cpu().numpy(), out)
    # the call's O0, recomputed on the host, reproduces it as an explicit h2_init
    assert m.last_hidden_call == 2
    again = ref.build(x, 69, h2_init=_cuda(m.hidden_draw())).cpu().numpy()
    assert np.array_equal(again, out)


def test_circuit_default_hidden_is_a_fresh_device_draw():
    mp = pkg()
    W = mp.weights
    meta = golden_meta()["circuit_s5_t3"]
    n, h, w, ssf, T = meta["n"], meta["h"], meta["w"], meta["ssf"], meta["timesteps"]
    wts, X, _ = MG.circuit_inputs(n, h, w, ssf, T, meta["weight_seed"], meta["x_seed"], meta["o0_seed"])
    cc = mp.hgru_module.ContextualCircuit(_cuda(X), timesteps=T, SRF=1, SSN=ssf, SSF=ssf, aux=HGRU_POSE_AUX)
    o_a = cc.build(weights=wts)[0].cpu().numpy()
    o_b = cc.build(weights=wts)[0].cpu().numpy()
    assert not np.array_equal(o_a, o_b)
    for c, got in ((0, o_a), (1, o_b)):
        o0 = W.synth_hidden(X.shape, seed=cc.hidden_seed + c)
        cc2 = mp.hgru_module.ContextualCircuit(_cuda(X), timesteps=T, SRF=1, SSN=ssf, SSF=ssf, aux=HGRU_POSE_AUX)
        exp = cc2.build(weights=wts, h2_init=_cuda(o0))[0].cpu().numpy()
        assert np.array_equal(got, exp), c


def test_reference_stack_order():
    """reference_stack_order=True returns the reference's interleaved TensorArray stacks: the "O"
    stack holds O_t where T-1-t is even and I_t elsewhere (hgru_module.py:825, 897-914)."""
    mp = pkg()
    meta = golden_meta()["circuit_s5_t3"]
    n, h, w, ssf, T = meta["n"], meta["h"], meta["w"], meta["ssf"], meta["timesteps"]
    wts, X, O0 = MG.circuit_inputs(n, h, w, ssf, T, meta["weight_seed"], meta["x_seed"], meta["o0_seed"])
    aux = dict(HGRU_POSE_AUX, store_states=True)
    cc = mp.hgru_module.ContextualCircuit(_cuda(X), timesteps=T, SRF=1, SSN=ssf, SSF=ssf, aux=aux)
    _, wa, _ = cc.build(weights=wts, h2_init=_cuda(O0))
    _, wr, _ = cc.build(weights=wts, h2_init=_cuda(O0), reference_stack_order=True)
    sO, sI = wa["store_O"].cpu().numpy(), wa["store_I"].cpu().numpy()
    rO, rI = wr["store_O"].cpu().numpy(), wr["store_I"].cpu().numpy()
    for t in range(T):
        o_first = (T - 1 - t) % 2 == 0
        assert np.array_equal(rO[:, t], sO[:, t] if o_first else sI[:, t])
        assert np.array_equal(rI[:, t], sI[:, t] if o_first else sO[:, t])
    assert np.array_equal(rO[:, T - 1], sO[:, T - 1])      # the last entry is always O_T
