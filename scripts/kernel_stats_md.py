#!/usr/bin/env python3
"""rocprofv3 ``*_kernel_stats.csv`` (or the ``*_results.db`` its default rocpd output writes)
-> markdown table (for profiles/).

    python scripts/kernel_stats_md.py gpurun_out/prof/run_kernel_stats.csv "title" [notes] > profiles/x.md
"""
import csv
import sys


def from_db(path):
    """the kernel_stats.csv columns from the rocpd sqlite database (its `kernels` view)"""
    import sqlite3
    con = sqlite3.connect(path)
    q = ("select name, count(*), sum(end - start), min(end - start) from kernels group by name")
    out = [dict(Name=n, Calls=c, TotalDurationNs=t, MinNs=m) for n, c, t, m in con.execute(q)]
    tot = sum(r["TotalDurationNs"] for r in out) or 1
    for r in out:
        r["AverageNs"] = r["TotalDurationNs"] / r["Calls"]
        r["Percentage"] = 100.0 * r["TotalDurationNs"] / tot
    return out


def main():
    path, title = sys.argv[1], sys.argv[2]
    notes = sys.argv[3] if len(sys.argv) > 3 else ""
    rows = from_db(path) if path.endswith(".db") else list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    if notes:
        print(notes + "\n")
    print(f"Total kernel time {total / 1e6:.3f} ms.\n")
    print("| kernel | calls | total ms | avg us | min us | % |")
    print("|---|---|---|---|---|---|")
    for r in rows[:20]:
        name = r["Name"]
        if len(name) > 80:
            name = name[:80]
        print(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['MinNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} |")


if __name__ == "__main__":
    main()
