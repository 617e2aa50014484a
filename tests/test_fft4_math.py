"""The index algebra of the four-step FFT loop (monkey-pose_amd/csrc/k_fft4.hip), restated in numpy
and checked against numpy's FFT on the CPU: the 72-point column transform split as
y = 8 n1 + n2, fy = k1 + 9 k2 (row kernel: 9-point sums over n1; column kernel: twiddle W72^{n2 k1}
and 8-point sums over n2), its inverse, and the real 72-point row transforms through a 36-point
complex FFT (rfft72_fwd / rfft72_inv).  A wrong sign, twiddle or index map in the kernels' design
shows up here without a GPU; the kernels themselves are checked against the oracle on the GPU
(tests/test_gpu_parity.py, tests/test_gpu_states.py)."""
import numpy as np

W72 = lambda m: np.exp(-2j * np.pi * m / 72)


def _forward_four_step(x):
    """x: [72 rows, cols] (rows >= 64 zero) -> X[fy][cols] via the row / column kernel split."""
    Z = np.zeros((8, 9) + x.shape[1:], complex)
    for n2 in range(8):                                   # row kernel, row class n2
        for k1 in range(9):
            Z[n2, k1] = sum(x[8 * n1 + n2] * np.exp(-2j * np.pi * n1 * k1 / 9) for n1 in range(9))
    X = np.zeros((72,) + x.shape[1:], complex)
    for k1 in range(9):                                   # column kernel, class k1
        for k2 in range(8):
            X[k1 + 9 * k2] = sum(Z[n2, k1] * W72(n2 * k1) * np.exp(-2j * np.pi * n2 * k2 / 8) for n2 in range(8))
    return X


def _inverse_four_step(X):
    """X: [72 fy][cols] -> x[y][cols] = sum_fy X[fy] e^{+2 pi i y fy / 72} (unnormalised)."""
    Zp = np.zeros((8, 9) + X.shape[1:], complex)
    for k1 in range(9):                                   # column kernel: 8-point inverse, twiddle
        for n2 in range(8):
            Zp[n2, k1] = sum(X[k1 + 9 * k2] * np.exp(2j * np.pi * n2 * k2 / 8) for k2 in range(8)) * np.conj(W72(n2 * k1))
    x = np.zeros((72,) + X.shape[1:], complex)
    for n2 in range(8):                                   # row kernel: 9-point inverse
        for n1 in range(9):
            x[8 * n1 + n2] = sum(Zp[n2, k1] * np.exp(2j * np.pi * n1 * k1 / 9) for k1 in range(9))
    return x


def test_four_step_column_transform_and_inverse():
    rng = np.random.default_rng(0)
    x = np.zeros((72, 5), complex)
    x[:64] = rng.standard_normal((64, 5)) + 1j * rng.standard_normal((64, 5))
    X = _forward_four_step(x)
    assert np.abs(X - np.fft.fft(x, axis=0)).max() < 1e-10
    back = _inverse_four_step(X) / 72
    assert np.abs(back - x).max() < 1e-12


def _rfft72_fwd(x64):
    """k_fft4.hip rfft72_fwd: z[m] = x[2m] + i x[2m+1] (x[64..71] = 0), FFT36, split by W72^k."""
    x = np.zeros(72)
    x[:64] = x64
    z = np.fft.fft(x[0::2] + 1j * x[1::2])
    out = []
    for k in range(37):
        zk, zm = z[k % 36], z[(36 - k) % 36]
        E = (zk + np.conj(zm)) / 2
        O = (zk - np.conj(zm)) / 2j
        out.append(E + W72(k) * O)
    return np.array(out)


def _rfft72_inv(X37):
    """k_fft4.hip rfft72_inv: E[k] = X[k] + conj X[36-k], O[k] = (X[k] - conj X[36-k]) W72^{-k},
    z = IDFT36(E + iO) (unnormalised): x[2m] = Re z[m], x[2m+1] = Im z[m]."""
    E = np.array([X37[k] + np.conj(X37[36 - k]) for k in range(36)])
    O = np.array([(X37[k] - np.conj(X37[36 - k])) * np.conj(W72(k)) for k in range(36)])
    z = np.fft.ifft(E + 1j * O) * 36
    x = np.empty(72)
    x[0::2], x[1::2] = z.real, z.imag
    return x[:64]


def test_real_row_transforms_via_36_point_fft():
    rng = np.random.default_rng(1)
    x = rng.standard_normal(64)
    X = _rfft72_fwd(x)
    full = np.zeros(72)
    full[:64] = x
    assert np.abs(X - np.fft.rfft(full)).max() < 1e-10
    # inverse of a Hermitian half spectrum = sum over all 72 frequencies (unnormalised)
    assert np.abs(_rfft72_inv(X) / 72 - x).max() < 1e-12


def test_2d_conv_through_the_split_matches_direct():
    """One 15x15 SAME cross-correlation (one channel) through row transforms + the four-step column
    split + the per-frequency product, against the direct sum: the loop's whole algebra."""
    rng = np.random.default_rng(2)
    H = Wd = 64
    R = 7
    img = rng.standard_normal((H, Wd))
    ker = rng.standard_normal((15, 15))
    pad = np.pad(img, R)
    direct = np.array([[np.sum(pad[y:y + 15, x:x + 15] * ker) for x in range(Wd)] for y in range(H)])
    # G[fy][fx] = sum_{ky,kx} w[ky][kx] e^{-2 pi i (fy (R - ky) + fx (R - kx)) / 72} (cross-correlation
    # as a convolution with the flipped kernel), 1/72^2 folded in -- k_fft.hip spec_weights_kernel
    fy = np.arange(72)[:, None, None, None]
    fx = np.arange(37)[None, :, None, None]
    ky = np.arange(15)[None, None, :, None]
    kx = np.arange(15)[None, None, None, :]
    G = (ker[None, None] * np.exp(-2j * np.pi * (fy * (R - ky) + fx * (R - kx)) / 72)).sum((2, 3)) / 72 ** 2
    x = np.zeros((72, 72))
    x[:H, :Wd] = img
    rows = np.array([_rfft72_fwd(x[y, :64]) for y in range(72)])   # [72 y][37 fx]
    S = _forward_four_step(rows)                                   # [72 fy][37 fx]
    Y = G * S
    back_rows = _inverse_four_step(Y)                              # [72 y][37 fx]
    out = np.array([_rfft72_inv(back_rows[y]) for y in range(H)])
    assert np.abs(out - direct).max() / np.abs(direct).max() < 1e-12
