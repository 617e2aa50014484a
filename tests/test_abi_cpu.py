"""CPU: the C-ABI library loads, exports every function include/monkeypose.h declares, the ctypes
table matches the header, and the facades reject bad input before touching a GPU.  No compute
call is made here (there is no GPU in the build container)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from helpers import HGRU_POSE_AUX, ROOT, pkg

HEADER = os.path.join(ROOT, "include", "monkeypose.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(mp_[a-z0-9_]+)\s*\(", txt)))


def test_header_lists_entry_points():
    fns = header_functions()
    for f in ("mp_create", "mp_set_weight", "mp_finalize_weights", "mp_hgru_pose_fwd",
              "mp_hgru_circuit_fwd", "mp_last_error", "mp_destroy"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    mp = pkg()
    path = mp._lib.LIB_PATH
    assert os.path.exists(path), "build first: python -c 'import __graft_entry__ as g; g.build()'"
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (mp_[a-z0-9_]+)", out))
    missing = set(header_functions()) - exported
    assert not missing, missing


def test_ctypes_table_matches_header():
    mp = pkg()
    assert sorted(set(mp._lib._SIGS) | set(mp.monkeydetector._CROP_SIGS)) == header_functions()


def test_library_loads_and_reports():
    mp = pkg()
    lib = mp._lib.load()
    assert lib.mp_version() == (0 << 16) | 3
    assert isinstance(lib.mp_last_error(), bytes)     # thread-local; earlier tests may have set it
    assert lib.mp_create(0, 99, ctypes.byref(ctypes.c_void_p())) < 0    # bad model kind
    assert b"model_kind" in lib.mp_last_error()


def test_header_compiles_as_c():
    src = '#include "monkeypose.h"\nint main(void){ return MP_OK; }\n'
    p = subprocess.run(["gcc", "-x", "c", "-std=c99", "-Wall", "-Werror", "-fsyntax-only",
                        "-I", os.path.dirname(HEADER), "-"], input=src, text=True, capture_output=True)
    assert p.returncode == 0, p.stderr


def test_facades_validate_before_gpu():
    import torch
    mp = pkg()
    m = mp.hgru_pose.model()
    with pytest.raises(NotImplementedError):
        m.build(torch.zeros((1, 128, 128, 1)), 69, train_mode=True)
    with pytest.raises(TypeError):
        m.build(torch.zeros((1, 128, 128, 1)), 69)           # CPU tensor: no CPU fallback
    with pytest.raises(NotImplementedError):
        mp.hgru_module.ContextualCircuit(torch.zeros((1, 16, 32, 64)), timesteps=2)   # default aux
    cc = mp.hgru_module.ContextualCircuit(torch.zeros((1, 16, 32, 64)), timesteps=2, SSF=15,
                                          aux=HGRU_POSE_AUX)
    assert cc.SSF_ext == 15 and cc.p_shape == [15, 15, 64, 64]
    with pytest.raises(TypeError):
        cc.build()


def test_reference_defaults_preserved():
    mp = pkg()
    m = mp.hgru_pose.model()
    assert (m.SRF, m.SSN, m.SSF, m.timesteps, m._BATCH_NORM_EPSILON) == (1, 15, 15, 8, 1e-5)
    assert m.aux == {k: v for k, v in HGRU_POSE_AUX.items()}


def test_auto_dtype_resolution():
    mp = pkg()
    r = mp._lib.resolve_dtype
    assert r('auto', 64, 64) == 'fp32_fft' and r('auto', 32, 32) == 'fp32_fft'
    assert r('auto', 16, 32) == 'fp32_fft'
    assert r('auto', 96, 96) == 'fp32_split' and r('auto', 50, 50) == 'fp32'
    assert r('fp32', 64, 64) == 'fp32'
    assert mp.hgru_pose.model().compute_dtype == 'auto'


@pytest.mark.gpu
def test_plain_c_client_matches_python(tmp_path):
    """tools/abi_demo.c (built by build() next to the .so) drives the ABI from C with hipMalloc'd
    buffers and no torch; its output equals the ctypes façade's bit for bit."""
    import subprocess
    torch = pytest.importorskip("torch")
    P = pkg()
    W = P.weights
    demo = os.path.join(os.path.dirname(P._lib.LIB_PATH), "abi_demo")
    assert os.path.exists(demo), "abi_demo not built (run __graft_entry__.build())"
    n, crop = 2, 64
    table = W.hgru_pose_vars(output_shape=69, timesteps=8, crop=crop)
    wts = {v.name: W.synth_value(v, 1234, 8) for v in table}
    depth = W.synth_crops(n, seed=42, size=crop)
    o0 = W.synth_hidden((n, crop // 2, crop // 2, 64), seed=7)
    with open(tmp_path / "manifest.txt", "w") as f:
        f.write(f"{n} {crop} {crop} 69 {P._lib.MP_DTYPE_F32_FFT}\n")
        for v in table:
            f.write(f"{v.name} {len(v.shape)} {' '.join(str(d) for d in v.shape)}\n")
    with open(tmp_path / "weights.bin", "wb") as f:
        for v in table:
            f.write(np.ascontiguousarray(wts[v.name], np.float32).tobytes())
    depth.astype(np.float32).tofile(tmp_path / "depth.bin")
    o0.astype(np.float32).tofile(tmp_path / "o0.bin")
    r = subprocess.run([demo, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = np.fromfile(tmp_path / "out.bin", np.float32).reshape(n, 69)
    m = P.hgru_pose.model()
    m.load_weights(wts)
    m.compute_dtype = "fp32_fft"
    ref = m.build(torch.from_numpy(depth).cuda(), 69, h2_init=torch.from_numpy(o0).cuda()).cpu().numpy()
    assert np.array_equal(got, ref)


def test_fwd_opts_struct_size_is_checked():
    """mp_fwd_opts (ABI 0.2) carries struct_size; a caller whose struct is smaller than the 0.2
    layout is rejected before anything is read past it (no GPU call: the check precedes the
    context)."""
    mp = pkg()
    L = mp._lib
    lib = L.load()
    assert ctypes.sizeof(L.FwdOpts) == 56 and ctypes.sizeof(L.PoseTaps) == 7 * 8   # the header layouts
    o = L.fwd_opts(L.MP_HIDDEN_RANDOM, 7, 0)
    o.struct_size = 16
    rc = lib.mp_hgru_pose_fwd_ex(None, None, 1, 128, 128, None, None, ctypes.byref(o), None)
    assert rc == -1 and b"struct_size" in lib.mp_last_error()
    rc = lib.mp_hgru_circuit_fwd_opts(None, None, None, 1, 64, 64, 64, 8, None, ctypes.byref(o), None)
    assert rc == -1 and b"struct_size" in lib.mp_last_error()
