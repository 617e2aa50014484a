"""HBM vs Infinity-Cache streaming rates: mp_hbm_probe over buffer sizes from 64 MiB (both buffers
of a copy inside the 256 MiB Infinity Cache) to 2 GiB (far past it)."""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mp = importlib.import_module("monkey-pose_amd")
for mib in (64, 96, 128, 256, 512, 2048):
    r = mp._lib.hbm_probe(0, mib << 20)
    print(json.dumps({"buffer_MiB": mib, **{k: v for k, v in r.items() if k.endswith("GBps")},
                      "forms": {k: v for k, v in r.items() if k.endswith("form")}}), flush=True)
