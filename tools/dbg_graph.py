import sys, os, importlib
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch
mode = sys.argv[1]
import test_dense_hier as T
if mode == "small":
    T.test_graph_runtime_small_graph(); print("small ok")
else:
    os.environ["MP_GRAPH_EXEC"] = mode
    m = T.golden_meta()["dense_hier_c128"]
    wts, depth = T.MG.regressor_inputs("dense_hier", 2, 128, m["weight_seed"], m["crop_seed"])
    model = T._gpu_model("fp32_split", wts)
    out = model.build(torch.from_numpy(depth).cuda(), *T.HEADS).cpu().numpy()
    print("err", T.rel_inf(out, T.golden_array("dense_hier_c128", "out")))
