"""Host-side pieces of config 5 on this machine's CPU: the native CoM crop of one 424x512 frame
(crop_batch, one thread) and getAbsoluteCoordinates, median microseconds."""
import importlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mp = importlib.import_module("monkey-pose_amd")
md = mp.monkeydetector.MonkeyDetector(365.456, 365.456, 256, 212, [800, 800, 1200], 200, 10000)
fr = list(mp.weights.synth_frames(8, seed=14)[..., 0] * np.float32(10000.0))
buf = np.empty((1, 128, 128, 1), np.float32)


def med(f, n=300):
    ts = []
    for i in range(n):
        t0 = time.perf_counter()
        f(i)
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts[30:])) * 1e6, 1)


com = np.array([256.0, 212.0, 1000.0])
rel = np.zeros((23, 3), np.float32)
print({"crop_batch_us": med(lambda i: md.crop_batch(fr[i % 8][None], None, nthreads=1, out=buf)),
       "center_of_mass_us": med(lambda i: md.calculateCoM(fr[i % 8])),
       "getAbsoluteCoordinates_us": med(lambda i: md.getAbsoluteCoordinates(rel, com))})
