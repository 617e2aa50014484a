"""Kernel statistics (the rocprofv3 --stats CSV columns) from a rocprofv3 SQLite (rocpd) database,
for runs whose profiler wrote only the .db:  python tools/rocpd_stats.py run_results.db > stats.csv"""
import collections
import csv
import sqlite3
import sys


def main(path):
    db = sqlite3.connect(path)
    q = ("select s.display_name, d.end - d.start from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    dur = collections.defaultdict(list)
    for name, ns in db.execute(q):
        dur[name].append(ns)
    total = sum(sum(v) for v in dur.values()) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), round(sum(v) / len(v), 3), round(100.0 * sum(v) / total, 2), min(v), max(v)])


if __name__ == "__main__":
    main(sys.argv[1])
