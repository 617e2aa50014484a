import importlib, os, sys, subprocess, numpy as np
sys.path.insert(0, os.getcwd())
code = r'''
import importlib, sys, os, numpy as np, torch
sys.path.insert(0, os.getcwd())
mp = importlib.import_module("monkey-pose_amd")
W = mp.weights
m = mp.train_hier_networks.hier_model_struct()
m.load_weights({v.name: W.synth_value(v, 5) for v in W.hier_vars()})
x = torch.from_numpy(W.synth_crops(256, seed=3, size=128)).cuda()
out = m.build(x, 108, 39, 39, 39, 39, 36).cpu().numpy()
np.save(sys.argv[1], out)
'''
for v in ("0", "1"):
    subprocess.run([sys.executable, "-c", code, f"/tmp/ts{v}.npy"], env=dict(os.environ, MP_IGEMM_TAPSKIP=v), check=True)
a, b = np.load("/tmp/ts0.npy"), np.load("/tmp/ts1.npy")
print("tapskip bit-identical:", np.array_equal(a, b), float(np.abs(a - b).max()))
