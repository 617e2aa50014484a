"""Write profiles/TREE_STAMP.json: the git head, whether the working tree differs from it, and the
source hash (bench.tree_stamp) of the tree about to be sent to a GPU box.  Profiling scripts copy it
next to the counters they collect (STAMP.json), and bench.py compares it with the tree it runs on.
usage (this container, before gpurun): python tools/stamp_tree.py"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv = sys.argv[:1]
import bench  # noqa: E402

head = subprocess.run(["git", "rev-parse", "HEAD"], cwd=ROOT, capture_output=True, text=True).stdout.strip()
dirty = subprocess.run(["git", "status", "--porcelain", "--", "monkey-pose_amd/csrc", "include"], cwd=ROOT,
                       capture_output=True, text=True).stdout.strip()
st = {"git_head": head, "native_sources_dirty": bool(dirty), "src_sha": bench.tree_stamp()}
with open(os.path.join(ROOT, "profiles", "TREE_STAMP.json"), "w") as f:
    json.dump(st, f, indent=1)
print(json.dumps(st))
