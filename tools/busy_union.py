"""GPU occupancy of the LAST pipeline run in a rocprofv3 kernel trace: the union of the kernel
intervals (time with at least one kernel on the device) against the span, the time with 2+
kernels overlapping, and the longest idle gaps (host round trips with no kernel queued).
usage: python3 tools/busy_union.py <trace_dir>"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    f = glob.glob(d + '/**/*kernel_trace.csv', recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
    ti = [i for i, r in enumerate(rows) if 'table_insert' in r['Kernel_Name']]
    run = rows[max(0, ti[-1] - 5):] if ti else rows
    ev = []
    for r in run:
        ev.append((int(r['Start_Timestamp']), 1))
        ev.append((int(r['End_Timestamp']), -1))
    ev.sort()
    t0, t1 = ev[0][0], ev[-1][0]
    depth, last, busy, multi, gaps = 0, t0, 0, 0, []
    for t, d_ in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            multi += t - last
        if depth == 0 and t > last:
            gaps.append(t - last)
        depth += d_
        last = t
    gaps.sort(reverse=True)
    print(f'span {(t1 - t0) / 1e6:.1f} ms, busy (>=1 kernel) {busy / 1e6:.1f} ms, overlapped (>=2) {multi / 1e6:.1f} ms, '
          f'idle {(t1 - t0 - busy) / 1e6:.1f} ms in {len(gaps)} gaps; longest gaps (us): '
          + ', '.join(f'{g / 1e3:.0f}' for g in gaps[:15]))


if __name__ == '__main__':
    main()
