"""Collect one tools/r6_final.sh run (gpurun_out/<tag>, parts A and B) into a committed profile
directory: rocprofv3 kernel stats, PMC bytes per dispatch (FETCH_SIZE x2 + WRITE_SIZE) and per forward,
MFMA-busy / stall shares, the bench line, the test log and the tree stamp they were taken on.
usage: python tools/r6_collect.py gpurun_out/<tag> profiles/r6"""
import glob
import json
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(*args):
    return subprocess.run([sys.executable, *args], capture_output=True, text=True, check=True, cwd=ROOT).stdout


def one(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        raise SystemExit(f"missing: {pattern}")
    return hits[0]


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    sa, sb = (json.load(open(os.path.join(src, f"STAMP_{p}.json"))) for p in "AB")
    if sa["src_sha"] != sb["src_sha"]:
        raise SystemExit(f"parts A and B ran on different trees: {sa} {sb}")
    json.dump(dict(sb, collected_from=src), open(os.path.join(dst, "STAMP.json"), "w"), indent=1)
    for f in ("bench_full_fp32.json", "gpu_tests.log"):
        shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    for d, tag in (("f32_fft", "fp32"), ("bf16", "bf16")):
        shutil.copy(one(f"{src}/kt_{d}/**/*kernel_stats.csv"), os.path.join(dst, f"kernel_stats_{tag}_1stream.csv"))
        fe = one(f"{src}/pmc_{d}_FETCH_SIZE/**/*counter_collection.csv")
        wr = one(f"{src}/pmc_{d}_WRITE_SIZE/**/*counter_collection.csv")
        open(os.path.join(dst, f"pmc_traffic_{tag}_b256.csv"), "w").write(run("tools/pmc_bytes.py", fe, wr))
        open(os.path.join(dst, f"pmc_forward_bytes_{tag}_1stream.txt"), "w").write(
            run("tools/pmc_forward_raw.py", fe, wr))
    fe = one(f"{src}/pmc2s_FETCH_SIZE/**/*counter_collection.csv")
    wr = one(f"{src}/pmc2s_WRITE_SIZE/**/*counter_collection.csv")
    open(os.path.join(dst, "pmc_traffic_fp32_b256_2stream.csv"), "w").write(run("tools/pmc_bytes.py", fe, wr))
    open(os.path.join(dst, "pmc_forward_bytes_fp32_2stream.txt"), "w").write(run("tools/pmc_forward_raw.py", fe, wr))
    mf = one(f"{src}/mfma/pose_f32_fft/**/*counter_collection.csv")
    open(os.path.join(dst, "mfma_util_pose_fp32_b256.csv"), "w").write(run("tools/pmc_mfma.py", mf))

    def forward_gb(path, first=None):
        """median GB per forward over the pass's forwards (first: only the first `first` of them -- the
        two-stream pass runs bench.py --steps 2 --warmup 1 on the default schedule, then its one-stream
        HIP-event profile pass)"""
        vals = [float(m.group(1)) for m in re.finditer(r"\]\s+([0-9.]+) GB", open(path).read())]
        vals = sorted(vals[:first] if first else vals)
        return vals[len(vals) // 2] if vals else None

    fw = {"source": f"tools/pmc_forward_raw.py over {src} (tools/r6_final.sh): FETCH_SIZE x2 + WRITE_SIZE per "
                    "dispatch, summed per pose forward (B = 256), one-time work excluded; median over the "
                    "forwards of the pass",
          "f32_fft": {"one_stream_GB": forward_gb(os.path.join(dst, "pmc_forward_bytes_fp32_1stream.txt")),
                      "two_stream_default_GB": forward_gb(os.path.join(dst, "pmc_forward_bytes_fp32_2stream.txt"), 3),
                      "files": [f"{dst}/pmc_forward_bytes_fp32_1stream.txt", f"{dst}/pmc_forward_bytes_fp32_2stream.txt"]},
          "bf16": {"one_stream_GB": forward_gb(os.path.join(dst, "pmc_forward_bytes_bf16_1stream.txt")),
                   "files": [f"{dst}/pmc_forward_bytes_bf16_1stream.txt"]}}
    json.dump(fw, open(os.path.join(dst, "pmc_forward_bytes.json"), "w"), indent=1)
    print(json.dumps(fw, indent=1))


if __name__ == "__main__":
    main()
