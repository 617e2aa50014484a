"""Summed PMC HBM bytes per pose forward, forward by forward, from the raw rocprofv3 counter CSVs of
a FETCH_SIZE pass and a WRITE_SIZE pass of the same bench command (tools/r5_final.sh pmc2s_*): the
dispatches are cut into forwards at each conv1_pool_bn_kernel (the backbone's first kernel), and
each forward is labelled by its column-kernel grid (a two-stream forward's hGRU launches carry half
the batch).  FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md); both counters in KB.
usage: python tools/pmc_forward_raw.py fetch.csv write.csv"""
import collections
import csv
import sys


def load(path, ctr):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == ctr:
            k = int(r["Dispatch_Id"])
            out[k] = (r["Kernel_Name"], int(r["Grid_Size"]), out.get(k, (0, 0, 0.0))[2] + float(r["Counter_Value"]))
    return out


def main():
    f = load(sys.argv[1], "FETCH_SIZE")
    w = load(sys.argv[2], "WRITE_SIZE")
    fwd, cur, seen_fc = [], None, True
    for d in sorted(f):
        name, grid, fv = f[d]
        # a forward starts at the first backbone kernel after the previous forward's fc_1 (with the
        # backbone per batch slice, each slice's backbone starts with conv1_pool_bn)
        if "conv1_pool_bn" in name and seen_fc:
            cur = collections.defaultdict(float)
            cur["_grids"] = set()
            fwd.append(cur)
            seen_fc = False
        if "fc_gemm" in name:
            seen_fc = True
        if cur is None or any(t in name for t in ("probe_", "rocclr", "at::native")):
            continue
        mb = (2 * fv + (w[d][2] if d in w else 0.0)) / 1e3
        key = name.split("(")[0][-40:]
        cur[key] += mb
        if "col8" in name or "spec_gemm" in name:
            cur["_grids"].add(grid)
    for i, c in enumerate(fwd):
        tot = sum(v for k, v in c.items() if not k.startswith("_"))
        print(f"forward {i}: col grids {sorted(c['_grids'])}  {tot / 1e3:.2f} GB")
        for k, v in sorted(((k, v) for k, v in c.items() if not k.startswith("_")), key=lambda kv: -kv[1])[:6]:
            print(f"    {v:9.1f} MB  {k}")


if __name__ == "__main__":
    main()
