"""CPU: variable tables (TF names / shapes / parameter counts) and the deterministic generators."""
import numpy as np

from helpers import pkg


def test_param_counts_match_survey():
    W = pkg().weights
    pose = W.hgru_pose_vars()
    total = sum(int(np.prod(v.shape)) for v in pose)
    assert total == 269_517_133                       # SURVEY.md 8d / BASELINE.md
    circ = W.hgru_circuit_vars()
    assert sum(int(np.prod(v.shape)) for v in circ) == 930_312
    names = [v.name for v in pose]
    assert len(names) == len(set(names))
    assert "cnn/contextual_circuit/p_r" in names and "cnn/fc_1/fc_1_weights" in names
    assert "cnn/batch_normalization_4/moving_variance" in names


def test_generator_is_deterministic_and_bounded():
    W = pkg().weights
    a = W.uniform01(1, "x", 1000)
    b = W.uniform01(1, "x", 1000)
    c = W.uniform01(2, "x", 1000)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert a.min() >= 0 and a.max() < 1 and abs(a.mean() - 0.5) < 0.05
    # chunking does not change the stream
    d = W.uniform01(1, "x", 1000, chunk=7)
    assert np.array_equal(a, d)


def test_synth_values():
    W = pkg().weights
    wts = W.synth_weights(W.hgru_circuit_vars(timesteps=8), seed=3)
    ib = wts["cnn/contextual_circuit/i_b"]
    ob = wts["cnn/contextual_circuit/o_b"]
    assert np.allclose(ob, -ib)                      # o_b = -i_b (hgru_module.py:386)
    assert (-ib >= 0).all() and (-ib <= np.log(7) + 1e-6).all()   # -log U(1, T-1)
    assert np.array_equal(wts["cnn/contextual_circuit/rho"], np.ones(8, np.float32))
    p = wts["cnn/contextual_circuit/p_r"]
    assert p.dtype == np.float32 and np.abs(p).max() <= W.glorot_limit(p.shape)


def test_synth_crops():
    W = pkg().weights
    c = W.synth_crops(3, seed=1, size=64)
    assert c.shape == (3, 64, 64, 1) and c.dtype == np.float32
    assert set(np.unique(c[c >= 0.999])) == {1.0}
    assert (c == 0).mean() > 0.02 and ((c > 0.19) & (c < 0.33)).mean() > 0.02
