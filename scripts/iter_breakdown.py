#!/usr/bin/env python3
"""Per-kernel time of one timed iteration from a rocprofv3 kernel trace (csv): the kernels
between the rollout launches number `which` and `which + 1` (diagnostics).

    python scripts/iter_breakdown.py gpurun_out/prof/run_kernel_trace.csv [which]
"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ro = [i for i, r in enumerate(rows) if "rollout_kernel" in r["Kernel_Name"]]
a, b = ro[which], ro[which + 1]
agg = defaultdict(lambda: [0, 0.0])
gaps, pe = 0, int(rows[a]["Start_Timestamp"])
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gaps += max(0, s - pe)
    pe = max(pe, e)
    k = r["Kernel_Name"][:90]
    agg[k][0] += 1
    agg[k][1] += (e - s) / 1e3
span = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
print(f"iteration {which}: span {span:.1f} us, idle gaps {gaps / 1e3:.1f} us")
print("| kernel | calls | total us | avg us |\n|---|---|---|---|")
for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"| `{k}` | {n} | {t:.1f} | {t / n:.1f} |")
