"""Structural pin of the hGRU oracle to the reference's own code (CPU, no GPU).

``tools/extract_hgru.py`` evaluates the reference's ``ContextualCircuit`` and ``hgru_pose.model``
method bodies (``hgru_module.py:9-959``, ``hgru_pose.py:8-216``) symbolically from their source
text; here the oracle (``oracle/hgru_ref.py``) is run on symbolic tensors (``tests/symbolic.py``)
and both expression DAGs are compared by Merkle hash: the oracle must apply the same ops, in the
same nesting, to the same named variables and inputs, for every timestep.  The oracle's conv /
pool / sigmoid primitives are swapped for symbolic ones here; their numerics are pinned by
``tests/test_oracle.py``.

Where /root/reference is absent (the GPU box), the committed digests
(``tests/golden/hgru_structure_digest.json``, written by ``--regen`` below from the reference)
stand in for it.
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import symbolic as S  # noqa: E402
from oracle import hgru_ref as R  # noqa: E402

DIGEST = os.path.join(ROOT, "tests", "golden", "hgru_structure_digest.json")
HAVE_REF = os.path.exists("/root/reference/hgru_module.py")
CIRCUIT_CASES = [  # (n, h, w, ssf, timesteps, hidden_init)
    (2, 16, 32, 15, 3, "random"),
    (2, 16, 32, 5, 2, "random"),
    (1, 32, 32, 15, 2, "zeros"),
    (1, 32, 32, 15, 2, "identity"),
]
POSE_CASE = (2, 128, 69)   # n, crop, output_shape (T = 8 from hgru_pose.model.__init__)


def _strip(name):
    return name[4:] if name.startswith("cnn/") else name


class SymWeights(dict):
    """the oracle's ``wts`` dict: every TF name maps to a symbolic variable (``cnn/`` dropped),
    shaped as the facade's weight table (``monkey-pose_amd/weights.py``) has it"""

    def __init__(self, table):
        super().__init__()
        self.shapes = {_strip(v.name): tuple(v.shape) for v in table}

    def __missing__(self, key):
        name = key[4:] if key.startswith("cnn/") else key
        return S.var(name, self.shapes.get(name))


@pytest.fixture
def symbolic_oracle(monkeypatch):
    monkeypatch.setattr(R, "conv2d_same", lambda x, w, stride=1: S.conv2d(x, w, stride, "SAME"))
    monkeypatch.setattr(R, "max_pool_same", lambda x, k=2, s=2: S.max_pool(x, k, s, "SAME"))
    monkeypatch.setattr(R, "sigmoid", S.sigmoid)
    return R


def _pkg():
    import importlib
    return importlib.import_module("monkey-pose_amd")


def _circuit_key(c):
    return "circuit_n{}_h{}_w{}_s{}_t{}_{}".format(*c)


def oracle_circuit(R_, case, o0_name):
    n, h, w, ssf, T, hidden_init = case
    X = S.inp("X", (n, h, w, 64))
    O0 = R_.hidden_init_state(X, hidden_init, S.inp(o0_name, (n, h, w, 64)))
    wts = SymWeights(_pkg().weights.hgru_circuit_vars(k=64, ssf=ssf, timesteps=T))
    O, steps, isteps = R_.hgru_forward(X, O0, wts, T, keep_inputs=True)
    return O, steps, isteps


def oracle_pose(R_, o0_name):
    n, crop, nout = POSE_CASE
    depth = S.inp("depth", (n, crop, crop, 1))
    O0 = S.inp(o0_name, (n, crop // 2, crop // 2, 64))
    table = _pkg().weights.hgru_pose_vars(output_shape=nout, timesteps=8, crop=crop)
    return R_.hgru_pose_forward(depth, SymWeights(table), O0, 8, np.float64)


def reference_digests():
    """{key: hash} of the reference's own expressions (needs /root/reference)"""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import extract_hgru as E
    out = {}
    for c in CIRCUIT_CASES:
        n, h, w, ssf, T, hi = c
        it, res, circ = E.circuit(n, h, w, ssf, T, hidden_init=hi, store_states=True)
        O, weights, _ = res
        assert O.op == "transpose" and O.args[1] == (1, 0, 2, 3, 4), "store_states stacks [n, T, ...]"
        o_steps = O.args[0].args[0]
        i_steps = weights["store_I"].items
        k = _circuit_key(c)
        out[k] = dict(O_stack=[s.h for s in o_steps], I_stack=[s.h for s in i_steps],
                      o0_input=f"rand#{it.rand_count - 1}", i0_input=f"rand#{it.rand_count - 2}",
                      free=sorted(S.free_inputs(o_steps[-1])), defects=it.defects)
        # store_states=False returns the last O itself (hgru_module.py:937-954)
        it2, res2, _ = E.circuit(n, h, w, ssf, T, hidden_init=hi, store_states=False)
        assert res2[0].h == o_steps[-1].h
    it, m = E.pose(*POSE_CASE)
    out["pose"] = dict(out_put=m.get("out_put", it).h, o0_input=f"rand#{it.rand_count - 1}",
                       free=sorted(S.free_inputs(m.get("out_put", it))), defects=it.defects,
                       weights=sorted(it.weights))
    return out


def _digest():
    with open(DIGEST) as f:
        return json.load(f)


@pytest.mark.parametrize("case", CIRCUIT_CASES, ids=_circuit_key)
def test_oracle_circuit_matches_reference_structure(symbolic_oracle, case):
    d = _digest()[_circuit_key(case)]
    O, steps, isteps = oracle_circuit(symbolic_oracle, case, d["o0_input"])
    T = case[4]
    # DEFECT 13: full(i0, O, I, store_O, store_I) (hgru_module.py:825) receives the loop vars
    # [i0, O, I, store_I, store_O] (897-908) and returns (..., store_I, store_O) (857), so the two
    # TensorArrays trade places every step: the reference's stacked "O" holds O_t where T-1-t is
    # even and I_t elsewhere (the last entry is always O_T).  The oracle keeps O_t and I_t apart.
    want_o = [(steps[t] if (T - 1 - t) % 2 == 0 else isteps[t]).h for t in range(T)]
    want_i = [(isteps[t] if (T - 1 - t) % 2 == 0 else steps[t]).h for t in range(T)]
    assert want_o == d["O_stack"], "per-step O_t / I_t differ from the reference's graph"
    assert want_i == d["I_stack"], "per-step I_t / O_t differ from the reference's graph"
    assert O.h == d["O_stack"][-1]
    # the reference's initial I draw never reaches the output (input_integration ignores it)
    assert d["i0_input"] not in d["free"]
    assert sorted(S.free_inputs(O)) == d["free"]


def test_oracle_pose_matches_reference_structure(symbolic_oracle):
    d = _digest()["pose"]
    out = oracle_pose(symbolic_oracle, d["o0_input"])
    assert out.h == d["out_put"], "hgru_pose_forward differs from hgru_pose.model.build's graph"
    assert sorted(S.free_inputs(out)) == d["free"]


def test_pose_resolves_exactly_the_surveyed_defects():
    d = _digest()["pose"]
    assert [x.split(":")[0] for x in d["defects"]] == ["1", "3", "5", "4"]


def test_pose_weight_names_are_the_facade_names(mp):
    """every variable the reference's build creates is one the facade's weight table names"""
    d = _digest()["pose"]
    table = mp.weights.hgru_pose_vars(output_shape=69, timesteps=8, crop=128)
    names = {_strip(v.name) for v in table}
    assert set(d["weights"]) == names


@pytest.mark.skipif(not HAVE_REF, reason="/root/reference not present (GPU box): digest only")
def test_digest_is_the_reference():
    assert reference_digests() == _digest()


def test_symbolic_canonical_form():
    a, b = S.inp("a", (1,)), S.inp("b", (1,))
    assert (a * b + 1).h == (1 + b * a).h
    assert (a - b).h == (a + (-1) * b).h
    assert (a * (b * 2)).h == ((a * 2) * b).h
    assert (a * b).h != (a + b).h
    assert S.tanh(a).h != S.sigmoid(a).h
    assert np.maximum(a, 0).h == S.relu(a).h


if __name__ == "__main__" and "--regen" in sys.argv:
    json.dump(reference_digests(), open(DIGEST, "w"), indent=1, sort_keys=True)
    print("wrote", DIGEST)
