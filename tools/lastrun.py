"""Per-kernel totals of the LAST pipeline run in a rocprofv3 kernel trace (the run starts at the
last screen table build), so warmup / setup dispatches do not blur a per-step view.
usage: python3 tools/lastrun.py <trace_dir> [top]"""
import collections, csv, glob, re, sys


def name(n):
    n = n.replace('(anonymous namespace)::', '').replace('void ', '')
    n = re.sub(r'\(.*', '', n)
    return n.split('::')[-1][:70]


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    f = glob.glob(d + '/**/*kernel_trace.csv', recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r['Start_Timestamp']))
    ti = [i for i, r in enumerate(rows) if 'table_insert' in r['Kernel_Name']]
    run = rows[max(0, ti[-1] - 5):] if ti else rows
    t = collections.Counter()
    c = collections.Counter()
    for r in run:
        k = name(r['Kernel_Name'])
        t[k] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        c[k] += 1
    span = (int(run[-1]['End_Timestamp']) - int(run[0]['Start_Timestamp'])) / 1e6
    busy = sum(t.values()) / 1e6
    print(f'last run: span {span:.1f} ms, dispatch time {busy:.1f} ms, {len(run)} dispatches')
    for k, v in t.most_common(top):
        print(f'{v / 1e6:9.1f} ms {c[k]:6d}  {k}')


if __name__ == '__main__':
    main()
