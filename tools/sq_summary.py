#!/usr/bin/env python3
"""SQ counter summary of the chaining kernel from tools/chain_pmc2.sh passes: per variant, the
counters summed over its chain_groups_kernel dispatches (the first pass of the real-anchor
dump), per 64 anchors, and the issue fractions of the CU's scalar unit and the SIMDs.

    python3 tools/sq_summary.py gpurun_out/r4b/pmc N_ANCHORS [variant ...]"""
import csv
import glob
import json
import os
import sys

CLK_GHZ = 2.4
N_CU = 256


def load(d):
    tot = {}
    disp = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "chain_groups_kernel<0>" not in r["Kernel_Name"]:
                continue
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            disp.setdefault(r["Counter_Name"], set()).add(r["Dispatch_Id"])
            disp.setdefault("_t", {})[r["Dispatch_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    return tot, disp


def main():
    d, n = sys.argv[1], float(sys.argv[2])
    names = sys.argv[3:] or sorted({os.path.basename(p).rsplit("_p", 1)[0] for p in glob.glob(os.path.join(d, "*_p1"))})
    out = {}
    for v in names:
        tot, disp = {}, {}
        for p in sorted(glob.glob(os.path.join(d, v + "_p*"))):
            if os.path.isdir(p):
                t, dd = load(p)
                nd = max(len(s) for k, s in dd.items() if k != "_t") if dd else 1
                for k, x in t.items():
                    tot[k] = x / nd    # per dispatch (the harness launches the kernel several times)
                disp.update(dd.get("_t", {}))
        per64 = {k: v_ * 64.0 / n for k, v_ in tot.items()}
        r = {"per_64_anchors": per64}
        if "SQ_INSTS_SALU" in tot and disp:
            ms = sum(e - s for s, e in disp.values()) / len(disp) / 1e6
            cyc = ms * 1e-3 * CLK_GHZ * 1e9
            r["kernel_ms"] = ms
            r["salu_issue_frac"] = tot["SQ_INSTS_SALU"] / (N_CU * cyc)            # 1 scalar unit per CU
            r["valu_issue_frac"] = tot["SQ_INSTS_VALU"] * 2 / (N_CU * 4 * cyc)     # wave64 VALU = 2 cycles, 4 SIMDs
        out[v] = r
        print(v, json.dumps({k: round(x, 1) for k, x in per64.items()}), {k: round(x, 3) for k, x in r.items() if k != "per_64_anchors"})
    return out


if __name__ == "__main__":
    main()
