#!/usr/bin/env python3
"""GPU idle gaps in a rocprofv3 kernel trace: the device timeline (kernels + copies merged
over every queue) from the last launch of MARK (default: the FASTA compaction kernel, the
first kernel of a bench step) to the end, its idle intervals longer than MIN_US, each with
the kernels on either side.

    python tools/gaps.py gpurun_out/iter/trace [MARK] [MIN_US]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("hymet::mm::", "")
    return n.split("(")[0][-60:]


def main():
    d = sys.argv[1]
    mark = sys.argv[2] if len(sys.argv) > 2 else "chunk_count_kernel"
    min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 200.0
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if mark in r[2]]
    if not starts:
        sys.exit(f"no kernel matching {mark}")
    rows = rows[starts[-1]:]
    t0, end = rows[0][0], rows[0][1]
    busy = 0
    gaps = []
    prev = rows[0][2]
    busy += rows[0][1] - rows[0][0]
    for s, e, n in rows[1:]:
        if s > end:
            gaps.append((s - end, prev, n))
        if e > end:
            busy += e - max(s, end)
            end = e
            prev = n
    span = end - t0
    idle = sum(g[0] for g in gaps)
    print(f"window {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms, idle {idle / 1e6:.1f} ms over {len(gaps)} gaps")
    by = defaultdict(lambda: [0, 0])
    for g, a, b in gaps:
        k = (short(a), short(b))
        by[k][0] += g
        by[k][1] += 1
    print("idle by (before -> after), top 40:")
    for (a, b), (g, c) in sorted(by.items(), key=lambda x: -x[1][0])[:40]:
        print(f"  {g / 1e6:8.2f} ms {c:6d}x  {a} -> {b}")
    big = [g for g in gaps if g[0] > min_us * 1e3]
    print(f"gaps > {min_us:.0f} us: {len(big)}, {sum(g[0] for g in big) / 1e6:.1f} ms")


if __name__ == "__main__":
    main()
