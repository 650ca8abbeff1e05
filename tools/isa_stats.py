#!/usr/bin/env python3
"""Static ISA statistics of one kernel in a hipcc -S output: instruction counts by class and
the register / spill / LDS metadata.  python3 tools/isa_stats.py FILE.s SYMBOL_SUBSTRING"""
import collections
import re
import sys


def stats(path, sym):
    t = open(path).read()
    m = re.search(r"^(_Z\S*" + re.escape(sym) + r"\S*):", t, re.M)
    a = m.end()
    b = t.index("s_endpgm", a)
    c = collections.Counter()
    for l in t[a:b].split("\n"):
        x = l.strip()
        if not x or x[0] in ";." or x.endswith(":"):
            continue
        op = x.split()[0]
        c["salu" if op.startswith("s_") else "valu" if op.startswith("v_") else "lds" if op.startswith("ds_")
          else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "other"] += 1
    md = {}
    k = t.index(".name:           " + m.group(1)) if (".name:           " + m.group(1)) in t else t.rindex(m.group(1))
    blk = t[t.rfind("  - .", 0, k):t.find("  - .", k + 10) if t.find("  - .", k + 10) > 0 else len(t)]
    for key in ("sgpr_count", "vgpr_count", "sgpr_spill_count", "vgpr_spill_count", "group_segment_fixed_size",
                "private_segment_fixed_size"):
        mm = re.search(r"\." + key + r":\s+(\d+)", blk)
        if mm:
            md[key] = int(mm.group(1))
    return dict(c), md


if __name__ == "__main__":
    print(*stats(sys.argv[1], sys.argv[2]))
