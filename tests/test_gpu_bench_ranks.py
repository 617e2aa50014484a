"""The bench's multi-rank path on hardware (BASELINE.json's 1/2/4/8-GPU metric).

* ``python bench.py --gpus 2`` run as the driver runs it (no launcher around it) must start two
  ranks itself and report ``n_gpus == 2`` / ``ranks == 2``; a launcher whose world differs from
  ``--gpus`` must fail.  gloo as the backend, because both ranks share the box's one GPU (RCCL
  refuses two ranks per device).
* RCCL itself: a one-rank ``nccl`` process group drives ``parallel.broadcast_weights`` (the
  bench's one collective) on CUDA tensors, so the RCCL broadcast executes on the MI355X; the
  broadcast blob must come back unchanged and pack to the same context output as a local load.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--backend", "gloo", "--batch", "16", "--steps", "2", "--warmup", "1", "--no-extras",
         "--no-cpu-baseline", "--no-parity"]


def _env():
    return dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
                PYTHONUNBUFFERED="1")


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-3000:]
    return json.loads(lines[-1])


def test_bench_gpus2_launches_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL,
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 2 and rec["ranks"] == 2
    assert rec["backend"] == "gloo" and len(rec["devices"]) == 2
    assert rec["config"]["global_batch"] == 32 and rec["value"] > 0


def test_bench_world_mismatch_fails():
    # a launcher with one rank but --gpus 2: the rank must refuse (non-zero exit, no JSON line)
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "--gpus 2" in r.stderr


_RCCL_CHILD = r"""
import datetime, importlib, os, sys
import numpy as np, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
mp = importlib.import_module("monkey-pose_amd")
W, par = mp.weights, mp.parallel
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev,
                        timeout=datetime.timedelta(seconds=120))
assert dist.get_backend() == "nccl"
table = W.hgru_pose_vars(output_shape=69, timesteps=8, crop=64)
wts = {v.name: W.synth_value(v, 1234, 8) for v in table}
for dtype in ("fp32", "bf16"):
    info = {}
    flat, layout, secs = par.broadcast_weights(table, wts, dev, 0, 1, dtype=dtype, info=info)
    torch.cuda.synchronize()
    assert flat.is_cuda and info["bytes"] > 0
    host = flat.cpu().numpy()
    for name, shape, off, n in layout:
        if dtype == "fp32" or name != par.FC1_NAME:
            assert np.array_equal(host[off:off + n], np.asarray(wts[name], np.float32).reshape(-1)), name
    print("BCAST", dtype, info["bytes"], secs, flush=True)
t = torch.arange(1 << 20, dtype=torch.float32, device=dev)
dist.all_reduce(t)
torch.cuda.synchronize()
assert torch.equal(t, torch.arange(1 << 20, dtype=torch.float32, device=dev))
dist.destroy_process_group()
print("RCCL_OK", flush=True)
"""


def test_rccl_one_rank_broadcast_weights():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = _env()
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    r = subprocess.run([sys.executable, "-c", _RCCL_CHILD, ROOT], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "RCCL_OK" in r.stdout
    assert r.stdout.count("BCAST") == 2
