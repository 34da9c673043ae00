#!/usr/bin/env python3
"""rocprofv3 kernel-trace database (rocpd SQLite) → kernel_stats CSV in rocprofv3's --stats layout.

    python tools/prof_summary.py gpurun_out/<dir>/run_results.db > profiles/<name>_kernel_stats.csv
"""
import csv
import math
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = {}
    for name, dur, vgpr, agpr, sgpr, lds, gx, wx in c.execute(
            "select name, duration, vgpr_count, accum_vgpr_count, sgpr_count, lds_size, grid_x, "
            "workgroup_x from kernels"):
        rows.setdefault(name, []).append((dur, vgpr, agpr, sgpr, lds, gx, wx))
    total = sum(d for v in rows.values() for d, *_ in v)
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev",
                "VGPR", "AGPR", "SGPR", "LDS", "Grid", "Workgroup"])
    for name, v in sorted(rows.items(), key=lambda kv: -sum(d for d, *_ in kv[1])):
        ds = [d for d, *_ in v]
        n = len(ds)
        avg = sum(ds) / n
        sd = math.sqrt(sum((d - avg) ** 2 for d in ds) / n)
        _, vg, ag, sg, lds, gx, wx = v[0]
        w.writerow([name, n, sum(ds), round(avg, 3), round(100.0 * sum(ds) / total, 2), min(ds), max(ds),
                    round(sd, 3), vg, ag, sg, lds, gx, wx])


if __name__ == "__main__":
    main(sys.argv[1])
