#!/usr/bin/env python3
"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv (or every csv under a dir).

    python tools/kstats.py gpurun_out/iter [N] [REGEX]
"""
import csv
import glob
import os
import re
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    rx = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
    files = [path] if path.endswith(".csv") else glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    shown = 0.0
    for r in rows:
        if rx and not rx.search(r["Name"]):
            continue
        if top <= 0:
            break
        top -= 1
        t = float(r["TotalDurationNs"]) / 1e6
        shown += t
        name = re.sub(r"hymet::mm::\(anonymous namespace\)::|rocprim::ROCPRIM_\d+_NS::detail::", "", r["Name"])
        print(f"{t:9.1f} ms {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f} us  {name[:110]}")
    print(f"shown {shown:.1f} ms of {total / 1e6:.1f} ms kernel time")


if __name__ == "__main__":
    main()
