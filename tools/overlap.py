"""Concurrency of the LAST pipeline run in a rocprofv3 kernel trace of the two-stream bench: per
kernel name, its summed duration, the part of it during which it ran alone on the device, and
the part shared with each other top kernel -- which kernels actually co-run and which hold the
device by themselves.  usage: python3 tools/overlap.py <trace_dir> [top]"""
import collections
import csv
import glob
import re
import sys


def name(n):
    n = n.replace('(anonymous namespace)::', '').replace('void ', '')
    n = re.sub(r'\(.*', '', n)
    return n.split('::')[-1][:40]


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    f = glob.glob(d + '/**/*kernel_trace.csv', recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
    ti = [i for i, r in enumerate(rows) if 'table_insert' in r['Kernel_Name']]
    run = rows[max(0, ti[-1] - 5):] if ti else rows
    ev = []
    for k, r in enumerate(run):
        ev.append((int(r['Start_Timestamp']), 1, k))
        ev.append((int(r['End_Timestamp']), -1, k))
    ev.sort()
    names = [name(r['Kernel_Name']) for r in run]
    alone = collections.Counter()
    pair = collections.Counter()
    total = collections.Counter()
    active = set()
    last = ev[0][0]
    for t, s, k in ev:
        dt = t - last
        if dt > 0 and active:
            act = sorted(active)
            for a in act:
                total[names[a]] += dt
            if len(act) == 1:
                alone[names[act[0]]] += dt
            else:
                for a in act:
                    for b in act:
                        if a != b:
                            pair[(names[a], names[b])] += dt / (len(act) - 1)
        if s > 0:
            active.add(k)
        else:
            active.discard(k)
        last = t
    tops = [k for k, _ in total.most_common(top)]
    print(f'{"kernel":40s} {"total":>8s} {"alone":>8s}  shared with (ms)')
    for k in tops:
        partners = sorted(((pair[(k, o)], o) for o in set(n for (a, n) in pair if a == k)), reverse=True)[:4]
        print(f'{k:40s} {total[k] / 1e6:8.1f} {alone[k] / 1e6:8.1f}  ' +
              ', '.join(f'{o} {v / 1e6:.1f}' for v, o in partners))


if __name__ == '__main__':
    main()
