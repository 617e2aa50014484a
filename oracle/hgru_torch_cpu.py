"""CPU BASELINE -- test infrastructure only (the import rule of oracle/hgru_ref.py applies).

A torch-CPU fp32 restatement of ``hgru_pose.model.build`` (``/root/reference/hgru_pose.py:47-105``;
the hGRU step of ``hgru_module.py:825-857`` exactly as ``oracle/hgru_ref.py::hgru_step`` states it),
the reference's TF-CPU path as BASELINE.md's CPU-baseline plan describes it: fp32, NHWC in / out,
``torch.nn.functional.conv2d`` on all the threads the process may use (oneDNN), timed by
``bench.py``'s ``cpu_baseline`` leg.  It is checked against the float64 numpy oracle in
``tests/test_oracle.py::test_torch_cpu_baseline_matches_oracle``.  Nothing in the product path
imports it.
"""
from __future__ import annotations

from typing import Dict

import numpy as np

BN_EPS = 1e-5


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))


def prepare(wts: Dict[str, np.ndarray], timesteps: int = 8):
    """The weights as torch CPU tensors in conv2d's OIHW layout, BN as (scale, shift)."""
    import torch
    P = {}

    def conv(name):   # HWIO -> OIHW
        return _t(wts[name]).permute(3, 2, 0, 1).contiguous()

    def bn(scope):
        g, b = _t(wts[f"{scope}/gamma"]), _t(wts[f"{scope}/beta"])
        m, v = _t(wts[f"{scope}/moving_mean"]), _t(wts[f"{scope}/moving_variance"])
        s = g / torch.sqrt(v + BN_EPS)
        return s, b - m * s

    for k in ("1", "2", "3"):
        P[f"c{k}w"] = conv(f"cnn/conv_{k}/conv_{k}_filters")
        P[f"c{k}b"] = _t(wts[f"cnn/conv_{k}/conv_{k}_biases"])
    for i, sc in enumerate(("cnn/batch_normalization", "cnn/batch_normalization_1", "cnn/batch_normalization_2",
                            "cnn/batch_normalization_3", "cnn/batch_normalization_4")):
        P[f"bn{i}"] = bn(sc)
    cc = "cnn/contextual_circuit"
    P["p_r"], P["i_r"], P["o_r"] = conv(f"{cc}/p_r"), conv(f"{cc}/i_r"), conv(f"{cc}/o_r")
    for n in ("i_b", "o_b", "beta", "nu", "gamma", "kappa", "omega", "lateral_bias"):
        P[n] = _t(wts[f"{cc}/{n}"]).reshape(1, -1, 1, 1)
    P["rho"] = [float(r) for r in np.asarray(wts[f"{cc}/rho"], np.float32).reshape(-1)[:timesteps]]
    P["fc1w"], P["fc1b"] = _t(wts["cnn/fc_1/fc_1_weights"]), _t(wts["cnn/fc_1/fc_1_biases"])
    P["fcow"], P["fcob"] = _t(wts["cnn/fc_out/fc_out_weights"]), _t(wts["cnn/fc_out/fc_out_biases"])
    return P


def _bn(x, sb):   # NCHW, per channel
    s, b = sb
    return x * s.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)


def forward(depth: np.ndarray, P, O0: np.ndarray, timesteps: int = 8) -> np.ndarray:
    """depth [n, 128, 128, 1], O0 [n, 64, 64, 64] NHWC fp32 -> [n, output_shape]."""
    import torch
    import torch.nn.functional as F
    with torch.no_grad():
        x = _t(depth).permute(0, 3, 1, 2)
        c1 = F.relu(F.conv2d(x, P["c1w"], P["c1b"], padding=1))                     # 50
        p1 = _bn(F.max_pool2d(c1, 2, 2), P["bn0"])                                   # 51-60
        c2 = _bn(F.relu(F.conv2d(p1, P["c2w"], P["c2b"], padding=1)), P["bn1"])      # 61-70
        X = _bn(F.relu(F.conv2d(c2, P["c3w"], P["c3b"], padding=1)), P["bn2"])       # 71-80
        O = _t(O0).permute(0, 3, 1, 2)
        pad = P["p_r"].shape[-1] // 2
        for t in range(timesteps):                                                   # hgru_module.py:825-857
            g1 = torch.sigmoid(F.conv2d(O, P["i_r"]) + P["i_b"])
            P1 = F.conv2d(O * g1, P["p_r"], padding=pad) + P["lateral_bias"]
            I = torch.tanh(X - (P["beta"] * O + P["nu"]) * P1)
            g2 = torch.sigmoid(F.conv2d(I, P["o_r"]) + P["o_b"])
            e = P["gamma"] * (F.conv2d(I, P["p_r"], padding=pad) + P["lateral_bias"])
            S = torch.tanh(P["kappa"] * (I + e) + P["omega"] * (I * e))
            O = (g2 * O + (1 - g2) * S) * P["rho"][t]
        h = _bn(O, P["bn3"]).permute(0, 2, 3, 1).reshape(O.shape[0], -1)           # 82-90, NHWC flatten
        r1 = F.relu(h @ P["fc1w"] + P["fc1b"])                                       # 91-92
        s, b = P["bn4"]
        r1 = r1 * s + b                                                              # 95-103 (DEFECT 5)
        return (r1 @ P["fcow"] + P["fcob"]).numpy()                                  # 104-105 (DEFECT 4)
