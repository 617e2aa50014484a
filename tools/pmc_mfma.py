"""MFMA utilisation per kernel from a tools/pmc_mfma.sh pass: MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) (the gfx950 MfmaUtil of rocprofiler-sdk's counter_defs.yaml,
whose GRBM max over XCDs we approximate by the per-XCD mean of the summed CSV value), plus the
share of wave cycles spent waiting (s_waitcnt / barrier: SQ_WAIT_ANY) and issue-stalled
(SQ_WAIT_INST_ANY).  usage: python tools/pmc_mfma.py <pmc_counter_collection.csv> [substring ...]"""
import collections
import csv
import sys

SIMDS, XCDS = 1024, 8


def main():
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(sys.argv[1])):
        rows[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    keys = sys.argv[2:]
    print("kernel,dispatches,mfma_util,wait_frac,issue_stall_frac,active_frac")
    out = []
    for k, c in rows.items():
        if keys and not any(s in k for s in keys):
            continue
        n = len(c["GRBM_GUI_ACTIVE"])
        mean = {name: sum(v) / len(v) for name, v in c.items()}
        gui = mean.get("GRBM_GUI_ACTIVE", 0.0) / XCDS
        util = mean.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui * SIMDS) if gui else 0.0
        wc = mean.get("SQ_WAVE_CYCLES", 0.0)
        f = (lambda x: mean.get(x, 0.0) / wc if wc else 0.0)
        out.append((mean.get("GRBM_GUI_ACTIVE", 0.0), f'"{k[:80]}",{n},{util:.4f},{f("SQ_WAIT_ANY"):.3f},'
                                                        f'{f("SQ_WAIT_INST_ANY"):.3f},{f("SQ_ACTIVE_INST_ANY"):.3f}'))
    for _, line in sorted(out, key=lambda t: -t[0]):
        print(line)


if __name__ == "__main__":
    main()
