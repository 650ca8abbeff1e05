"""Kernel statistics from a rocprofv3 rocpd database (rocprofv3 --kernel-trace writes
`<name>_results.db` by default): the same columns as rocprofv3's kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [out.csv]
"""
import csv
import re
import sqlite3
import sys


def short(name):
    m = re.search(r"(\w+_kernel\w*|radix_sort_\w+|scan_\w+|\w+)(?:<[^()]*>)?\(", name)
    return m.group(1) if m else name[:80]


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, (end - start) from kernels").fetchall()
    agg = {}
    for name, d in rows:
        a = agg.setdefault(name, [0, 0, None, 0, 0.0])
        a[0] += 1
        a[1] += d
        a[2] = d if a[2] is None else min(a[2], d)
        a[3] = max(a[3], d)
        a[4] += float(d) * d
    total = sum(a[1] for a in agg.values()) or 1
    out = []
    for name, (n, tot, mn, mx, sq) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        avg = tot / n
        sd = max(0.0, sq / n - avg * avg) ** 0.5
        out.append([name, n, tot, avg, 100.0 * tot / total, mn, mx, sd])
    return out


def main():
    rows = stats(sys.argv[1])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w", newline="") as fh:
            w = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
            w.writerows(rows)
    for r in rows[:40]:
        print(f"{r[2]/1e6:10.1f} ms {r[1]:7d} calls {r[3]/1e3:10.1f} us avg {r[4]:5.1f}%  {short(r[0])}")


if __name__ == "__main__":
    main()
