"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv: one row per (kernel, counter),
the mean over dispatches (optionally only dispatches of a given grid size).
usage: python tools/pmc_summary.py <csv> [kernel-substring ...]"""
import csv
import sys
from collections import defaultdict

rows = defaultdict(list)
grids = {}
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        k = r["Kernel_Name"]
        short = k.split("(")[0].replace("void mp::", "").replace("mp::", "")
        key = (short, r["Grid_Size"])
        rows[(key, r["Counter_Name"])].append(float(r["Counter_Value"]))
want = sys.argv[2:]
out = defaultdict(dict)
for ((short, grid), ctr), v in rows.items():
    if want and not any(w in short for w in want):
        continue
    out[(short, grid)][ctr] = (sum(v) / len(v), len(v))
for (short, grid), d in sorted(out.items()):
    n = max(c for _, c in d.values())
    print(f"{short[:60]:60s} grid={grid:>8s} n={n:3d} " + " ".join(f"{c}={v:.4g}" for c, (v, _) in sorted(d.items())))

# busy fractions: counter / (CUs * mean duration * clock), --clock GHz (default 2.4)
if "--dur" in sys.argv[0:0]:
    pass
