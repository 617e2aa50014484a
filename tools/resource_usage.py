"""Per-kernel register / scratch / LDS / occupancy table of the HIP library, from the compiler's
-Rpass-analysis=kernel-resource-usage remarks (gfx950, the Makefile's flags per source).
usage: python tools/resource_usage.py > profiles/<tag>/kernel_resource_usage.txt"""
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "monkey-pose_amd", "csrc")
SOURCES = ["k_fft.hip", "k_fc.hip", "k_igemm.hip", "k_conv64x3.hip", "k_conv64.hip", "k_frame.hip"]
FIELDS = ["VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
    return out if len(out) == len(names) else names


def main():
    rows = []
    for src in SOURCES:
        extra = ["-fno-slp-vectorize"] if src == "k_fft.hip" else []
        cmd = ["/opt/rocm/bin/hipcc", *extra, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
               os.path.join(CSRC, src), "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
        err = subprocess.run(cmd, capture_output=True, text=True).stderr
        cur = None
        for line in err.splitlines():
            m = re.search(r"remark:\s+Function Name: (\S+)", line)
            if m:
                cur = {"src": src, "name": m.group(1)}
                rows.append(cur)
                continue
            for f in FIELDS:
                m = re.search(r"remark:\s+" + re.escape(f) + r": (\d+)", line)
                if m and cur is not None:
                    cur[f] = int(m.group(1))
    names = demangle([r["name"] for r in rows])
    print("source | kernel | VGPRs | AGPRs | scratch B/lane | waves/SIMD | LDS B/block")
    for r, n in zip(rows, names):
        print(" | ".join([r["src"], n[:150]] + [str(r.get(f, "")) for f in FIELDS]))


if __name__ == "__main__":
    sys.exit(main())
