"""Full-size oracle outputs of bench.py's CAMI workloads, generated once on the CPU with the
oracle restatements (TEST INFRASTRUCTURE: the checker's expected values, never the product):

    python tests/golden/make_cami_golden.py cami-medium   # C4: screen + PAF + TSV, every contig
    python tests/golden/make_cami_golden.py cami-high --screen-only   # C5: the three-DB screen

The workload is bench.cami_inputs (same seeds, same FASTA bytes, same decoys) with the DB
sketches computed by the oracle's Mash sketch instead of the GPU (the fixture records the
digest of every DB's hashes, and the GPU test asserts its own DBs hash the same).  Then
run_hymet_cami.sh's steps 1-5 on the oracle (oracle/pipeline_oracle.py): mash screen ->
mash.sh selection -> limit_candidates -> minimap2 -I2g -d / -x asm10 -> classification_cami.
Writes tests/golden/cami/<workload>.{json,npz} (tests/_digest.py)."""
import argparse
import os
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import bench  # noqa: E402
import _digest  # noqa: E402
from oracle import classify_oracle, oracle_lib, pipeline_oracle, select_oracle  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "cami")


def log(*a):
    print(f"[golden {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload", choices=["cami-medium", "cami-high"])
    ap.add_argument("--screen-only", action="store_true")
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--out", default=OUT)
    ap.add_argument("--bench-args", default="", help="extra bench.py arguments (trial runs on a smaller workload)")
    a = ap.parse_args()
    args = bench.parse_args(["--workload", a.workload] + a.bench_args.split())
    t00 = time.time()

    def oracle_sketch(w):
        with ThreadPoolExecutor(a.threads) as ex:
            return list(ex.map(lambda g: np.sort(oracle_lib.sketch([g], 21, 42, 1000)), w.refs))

    w, fasta, dbs = bench.cami_inputs(args, oracle_sketch)
    names = list(w.contig_names)
    index = _digest.name_index(names)
    seqs = list(w.contigs)
    meta = {"workload": a.workload, "contigs": len(names), "contig_bases": w.contig_bases,
            "fasta_sha256": _digest.sha(fasta), "db_hashes_sha256": [_digest.sha(d.hashes) for d in dbs],
            "db_refs": [d.n_refs for d in dbs]}
    del fasta
    arrays = {}
    # 1. mash screen, one run per DB (mash.sh:14), full shared / median arrays
    tabs = []
    for d, db in enumerate(dbs):
        t0 = time.time()
        so = oracle_lib.ScreenOracle(db)
        sh, md, ss, nk = so.run(seqs)
        del so
        arrays[f"screen{d}_shared"] = sh
        arrays[f"screen{d}_median"] = md
        meta[f"screen{d}_set_size"] = int(ss)
        meta[f"screen{d}_n_kmers"] = int(nk)
        refs = [(db.names[i], db.comments[i], int(db.offsets[i + 1] - db.offsets[i])) for i in range(db.n_refs)]
        rows = select_oracle.sort_gr(select_oracle.sort_unique_k5(select_oracle.screen_lines(refs, sh, md, ss, db.k)))
        tabs.append(rows)
        log(f"screen DB {d}: {db.n_refs} refs, {int((sh > 0).sum())} with hits, {len(rows)} rows ({time.time()-t0:.0f}s)")
    # 2-3. selection per DB, union, limit_candidates
    sels = [select_oracle.select_threshold(rows, "0.9", 1)[2] for rows in tabs]
    selected = select_oracle.union_sorted(*sels)
    scores = {}
    for rows in tabs:
        for line in rows:
            p = line.split("\t")
            try:
                s = float(p[0])
            except ValueError:
                continue
            if p[4] not in scores or s > scores[p[4]]:
                scores[p[4]] = s
    selected, _ = select_oracle.limit_candidates(selected, scores, args.cand_max)
    meta["selected"] = len(selected)
    meta["selected_sha256"] = _digest.sha("".join(n + "\n" for n in selected).encode())
    log(f"selected {len(selected)} candidates ({time.time()-t00:.0f}s)")
    if not a.screen_only:
        # 4. minimap2 -I2g -d + -x asm10 over every contig
        by_name = {n + ".fna.gz": i for i, n in enumerate(w.ref_names)}
        rn = [w.ref_names[by_name[n]] for n in selected]
        rs = [w.refs[by_name[n]] for n in selected]
        t0 = time.time()
        paf = pipeline_oracle.map_paf(rn, rs, list(zip(names, seqs)), threads=a.threads)
        log(f"mapped {len(names)} contigs: {len(paf)} PAF lines ({time.time()-t0:.0f}s)")
        paf_b = "".join(l + "\n" for l in paf).encode()
        del paf
        # 5. classification_cami.py
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "resultados.paf")
            with open(p, "wb") as f:
                f.write(paf_b)
            tax = os.path.join(td, "detailed_taxonomy.tsv")
            hier = os.path.join(td, "taxonomy_hierarchy.tsv")
            open(tax, "w").write(w.taxonomy_tsv())
            open(hier, "w").write(w.hierarchy_tsv())
            tsv = classify_oracle.classify_cami(p, tax, hier)
        cnt, dig = _digest.paf_digests(paf_b, index)
        tsv_sha, tdig, order = _digest.tsv_digests(tsv, index)
        arrays.update(paf_count=cnt, paf_digest=dig, tsv_digest=tdig, tsv_order=order)
        meta.update(paf_lines=int(cnt.sum()), paf_sha256=_digest.sha(paf_b), tsv_sha256=tsv_sha, tsv_rows=len(order))
    meta["oracle_seconds"] = round(time.time() - t00, 1)
    meta["threads"] = a.threads
    _digest.save(os.path.join(a.out, a.workload + ("-screen" if a.screen_only else "")), meta, arrays)
    log("wrote", meta)


if __name__ == "__main__":
    main()
