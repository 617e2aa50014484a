"""Summed PMC HBM bytes of ONE pose forward from a tools/pmc_bytes.py summary (per-kernel bytes per
dispatch x dispatches), without the one-time work in the same process (the HBM probe kernels, weight
packing, spectral-weight build): forwards counted as the column-kernel dispatches / 16 (two per
timestep, T = 8; the six-launch loop: spec_gemm likewise).  usage: python tools/pmc_forward.py
<pmc_traffic.csv> [per-forward-col-launches]"""
import csv
import sys

ONE_TIME = ("probe_", "pack_", "spec_weights", "absmax", "fill", "rocclr", "init_weights", "synth")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    per_fwd = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    col = [r for r in rows if "col8" in r["kernel"] or "spec_gemm" in r["kernel"]]
    nfwd = sum(int(r["dispatches"]) for r in col) / per_fwd
    out, tot = [], 0.0
    for r in rows:
        if any(t in r["kernel"] for t in ONE_TIME):
            continue
        mb = float(r["traffic_MB"]) * int(r["dispatches"]) / nfwd
        tot += mb
        out.append((mb, r["kernel"][:70], int(r["dispatches"]) / nfwd, float(r["traffic_MB"])))
    print(f"forwards in the pass: {nfwd:g}; summed HBM bytes per forward: {tot / 1e3:.2f} GB")
    for mb, k, n, per in sorted(out, reverse=True):
        if mb > 1:
            print(f"  {mb:9.1f} MB  {n:5.2f} launches x {per:8.1f} MB  {k}")


if __name__ == "__main__":
    main()
