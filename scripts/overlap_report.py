#!/usr/bin/env python3
"""Collective/compute overlap from a rocprofv3 kernel trace (``*_kernel_trace.csv``).

For every RCCL kernel (name contains "nccl" or "rccl") the time it shares with the compute
kernels running at the same moment on other queues/streams, per compute kernel name; plus the
median RCCL kernel duration and the share of it covered by compute.

    python scripts/overlap_report.py gpurun_out/x/run_kernel_trace.csv > profiles/r3/overlap.md
"""
import csv
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return name.split("(")[0][:70]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", r.get("Queue_Id")))
          for r in rows]
    coll = [k for k in ks if "nccl" in k[2].lower() or "rccl" in k[2].lower()]
    comp = [k for k in ks if k not in coll and not k[2].startswith("__amd_rocclr")]
    comp.sort()
    print("# RCCL / compute overlap (rocprofv3 kernel trace)\n")
    print(f"{len(coll)} collective kernels, {len(comp)} compute kernels.\n")
    if not coll:
        return
    covered, durs = [], []
    by_name = defaultdict(int)
    for s, e, n, st in coll:
        durs.append(e - s)
        # union of compute intervals inside [s, e]
        iv = sorted((max(s, cs), min(e, ce), cn) for cs, ce, cn, _ in comp if cs < e and ce > s)
        tot, cur_s, cur_e = 0, None, None
        for a, b, cn in iv:
            by_name[short(cn)] += b - a
            if cur_e is None or a > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = a, b
            else:
                cur_e = max(cur_e, b)
        if cur_e is not None:
            tot += cur_e - cur_s
        covered.append(tot / max(1, e - s))
    print(f"collective kernel duration: median {statistics.median(durs) / 1e3:.1f} us, "
          f"total {sum(durs) / 1e6:.3f} ms\n")
    print(f"share of collective time with a compute kernel running: median {statistics.median(covered):.2f}, "
          f"mean {statistics.mean(covered):.2f}\n")
    print("| compute kernel overlapping the collectives | overlap ms |")
    print("|---|---|")
    for n, t in sorted(by_name.items(), key=lambda x: -x[1])[:12]:
        print(f"| `{n}` | {t / 1e6:.3f} |")


if __name__ == "__main__":
    main()
