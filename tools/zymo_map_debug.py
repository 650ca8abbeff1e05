#!/usr/bin/env python3
"""GPU-box diagnostic: map the 322 re-cut Zymo contigs (tests/_zymo.py) against the 63 real
genome sequences with the GPU path and compare with the oracle PAF.

    python tools/zymo_map_debug.py OUTDIR [ENV=VAL ...]

The oracle PAF is computed once into OUTDIR/oracle.paf; the GPU PAF goes to
OUTDIR/gpu.paf; a summary line (lines, equal, first difference) is printed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out = sys.argv[1]
    for kv in sys.argv[2:]:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    os.makedirs(out, exist_ok=True)
    from tests import _zymo as z
    seqs = z.sequences()
    q = z.recut_queries()
    op = os.path.join(out, "oracle.paf")
    if os.environ.get("NO_ORACLE"):
        op = None
    elif not os.path.exists(op):
        from oracle import pipeline_oracle
        o = pipeline_oracle.map_paf([n for n, _ in seqs], [s for _, s in seqs], [(n, s) for n, s, _ in q], threads=16)
        with open(op, "w") as f:
            f.write("".join(l + "\n" for l in o))
    o_paf = open(op).read().splitlines() if op else []
    from hymet_amd import cli, ingest
    from hymet_amd._lib import Gpu
    from hymet_amd.seqio import from_records
    gpu = Gpu(0)
    refs = from_records([(n, "", s) for n, s in seqs])
    parts, names, lens, first = cli.build_parts(gpu, refs, "2g", 50e6)
    fasta = ingest.to_fasta([n for n, _, _ in q], [s for _, s, _ in q])
    paf = None
    for r in range(int(os.environ.get("REPEAT", "1"))):
        try:
            p2 = cli.map_paf(gpu, parts, names, lens, first, fasta).decode().splitlines()
        except Exception as e:  # noqa: BLE001
            print(f"[{' '.join(sys.argv[2:])}] run {r}: map failed: {e}", flush=True)
            continue
        if paf is not None:
            print(f"  run {r}: identical to run 0: {p2 == paf}", flush=True)
        else:
            paf = p2
    if paf is None:
        return 1
    with open(os.path.join(out, "gpu.paf"), "w") as f:
        f.write("".join(l + "\n" for l in paf))
    diff = next((i for i, (a, b) in enumerate(zip(paf, o_paf)) if a != b), None)
    print(f"[{' '.join(sys.argv[2:])}] gpu {len(paf)} oracle {len(o_paf)} equal {paf == o_paf} first_diff {diff}", flush=True)
    if diff is not None:
        print("  gpu   :", paf[diff], "\n  oracle:", o_paf[diff], flush=True)
    a = z.primary_agreement(q, paf)
    print("  agreement:", {k: v for k, v in a.items() if k != "misses"}, a["misses"], flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
