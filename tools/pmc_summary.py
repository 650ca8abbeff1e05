"""Per-launch HBM traffic of the bench's kernels from rocprofv3 PMC passes.

    rocprofv3 --pmc FETCH_SIZE --kernel-include-regex R --output-format csv -d D1 -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-include-regex R --output-format csv -d D2 -o run -- python3 bench.py ...
    python tools/pmc_summary.py OUT.json D1 D2

Writes {kernel symbol: {"dispatches", "fetch_kb", "write_kb", "traffic_bytes"}} averaged per
dispatch.  FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half of the bytes of
wide (16 B/lane) coalesced reads (MI355X_MICROARCH.md, HBM section), so traffic_bytes =
(2 * FETCH_SIZE + WRITE_SIZE) * 1024 -- an upper estimate of the read side for narrower loads.
"""
import csv
import glob
import json
import os
import re
import sys


def kernel_key(name: str) -> str:
    """'void ns::(anonymous namespace)::chain_groups_kernel<1>(Params)' -> 'chain_groups_kernel<1>'"""
    m = re.search(r"(\w+)(<[^()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name


def read_counters(d: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = {}
    for fn in files:
        with open(fn, newline="") as fh:
            for row in csv.DictReader(fh):
                k = kernel_key(row["Kernel_Name"])
                c = row["Counter_Name"]
                v = float(row["Counter_Value"])
                disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
                e = out.setdefault(k, {}).setdefault(c, {})
                e[disp] = e.get(disp, 0.0) + v  # counters summed over agents/dimensions per dispatch
    return out


def main():
    dst, dirs = sys.argv[1], sys.argv[2:]
    acc = {}
    for d in dirs:
        for k, cs in read_counters(d).items():
            for c, per in cs.items():
                a = acc.setdefault(k, {})
                a[c] = (sum(per.values()) / max(len(per), 1), len(per))
    res = {}
    for k, cs in acc.items():
        f = cs.get("FETCH_SIZE", (None, 0))
        w = cs.get("WRITE_SIZE", (None, 0))
        r = {"dispatches": max(f[1], w[1]), "fetch_kb": f[0], "write_kb": w[0]}
        if f[0] is not None and w[0] is not None:
            r["traffic_bytes"] = (2.0 * f[0] + w[0]) * 1024.0
        res[k] = r
    with open(dst, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    for k, r in sorted(res.items()):
        print(k, r)


if __name__ == "__main__":
    main()
