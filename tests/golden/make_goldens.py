#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ by running the REFERENCE
scripts themselves (importable in the build container only; never on the GPU box).

    python tests/golden/make_goldens.py  [--ref /root/reference]

What it writes (all small, all data -- inputs + expected outputs):
  classify/  zymo.paf (copy of case/truth/zymo_mc/zymo_mc_vs_refs.paf), taxonomy + hierarchy
             TSVs derived from case/truth/zymo_refs/seqid2taxid.tsv and
             case/truth/zymo_mc/truth_profile.cami.tsv (recipe: case/results_summary.md:132-156),
             synthetic edge-case PAFs, and the expected TSV bytes of
             scripts/classification_cami.py and scripts/classification.py for each combination.
  fallback/  expected outputs of tools/build_id_map.py and tools/mini_classify.py (the
             run_hymet_cami.sh:183-205 classification fallback) on the classify fixtures.
  limit/     synthetic screen tables + selected lists and the expected output of
             scripts/limit_candidates.py (offline flags only: never --dedupe without --no-download).
"""
from __future__ import annotations

import argparse
import contextlib
import csv
import importlib.util
import io
import json
import os
import random
import shutil
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent


def load_module(path: Path, name: str):
    spec = importlib.util.spec_from_file_location(name, str(path))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod  # Pool workers / dataclasses resolve the module by name
    spec.loader.exec_module(mod)
    return mod


def build_taxonomy_inputs(ref: Path, out: Path):
    seqmap = ref / "case/truth/zymo_refs/seqid2taxid.tsv"
    rows = [r for r in csv.reader(open(seqmap), delimiter="\t") if r]
    by_tax = {}
    for seq, tax in rows:
        by_tax.setdefault(tax, []).append(seq)
    with open(out / "zymo_taxonomy.tsv", "w") as f:
        f.write("GCF\tTaxID\tIdentifiers\n")
        for tax, seqs in sorted(by_tax.items(), key=lambda x: int(x[0])):
            f.write(f"ZymoTax_{tax}\t{tax}\t{';'.join(seqs)}\n")
    prof = ref / "case/truth/zymo_mc/truth_profile.cami.tsv"
    species = []
    for line in open(prof):
        if line.startswith(("#", "@")) or not line.strip():
            continue
        p = line.rstrip("\n").split("\t")
        if p[1] == "species":
            species.append(p)
    ranks = ["superkingdom", "phylum", "class", "order", "family", "genus", "species"]
    for label in ("domain", "superkingdom"):
        with open(out / f"zymo_hierarchy_{label}.tsv", "w") as f:
            f.write("TaxID\tName\tRank\tParentTaxID\tLineage\n")
            for p in species:
                taxids = p[2].split("|")
                names = p[3].split("|")
                lin = ";".join(f"{(label if r == 'superkingdom' else r)}:{n}" for r, n in zip(ranks, names))
                f.write(f"{p[0]}\t{names[-1]}\tspecies\t{taxids[-2]}\t{lin}\n")
    # a hierarchy exercising alias / k__ / plain-name / NA / override parsing paths
    with open(out / "mixed_hierarchy.tsv", "w") as f:
        f.write("TaxID\tName\tRank\tParentTaxID\tLineage\n")
        mix = [
            ("562", "domain:Bacteria;kingdom:Pseudomonadati;p:Pseudomonadota;c:Gammaproteobacteria;o:Enterobacterales;f:Enterobacteriaceae;g:Escherichia;s:Escherichia coli;strain:K-12"),
            ("28901", "k__Bacteria; p__Pseudomonadota; c__Gammaproteobacteria; o__Enterobacterales; f__Enterobacteriaceae; g__Salmonella; s__Salmonella enterica"),
            ("1423", "Bacteria;Bacillota;Bacilli;NA;Bacillaceae;Bacillus;Bacillus subtilis"),
            ("1280", "Bacteria|Bacillota|Bacilli|Bacillales|Staphylococcaceae|Staphylococcus|Staphylococcus aureus"),
            ("1639", "domain:Bacteria;phylum:Bacillota;class:Bacilli;order:Bacillales;family:Listeriaceae;genus:Listeria;species:Listeria monocytogenes"),
            ("1351", "domain:Bacteria;phylum:Bacillota;class:Bacilli;order:Lactobacillales;family:Enterococcaceae;genus:Enterococcus;species:Enterococcus faecalis"),
            ("1613", "domain:Bacteria;phylum:Bacillota;class:Bacilli;order:Lactobacillales;family:Lactobacillaceae;genus:Limosilactobacillus;species:Limosilactobacillus fermentum"),
            ("287", "domain:Bacteria;phylum:Pseudomonadota;class:Gammaproteobacteria;order:Pseudomonadales;family:Pseudomonadaceae;genus:Pseudomonas;species:Pseudomonas aeruginosa"),
            ("4932", "domain:Eukaryota;phylum:Ascomycota;class:Saccharomycetes;order:Saccharomycetales;family:Saccharomycetaceae;genus:Saccharomyces;species:Saccharomyces cerevisiae"),
            ("5207", "domain:Eukaryota;unknownrank:x;phylum:;class:Tremellomycetes"),
        ]
        for tid, lin in mix:
            f.write(f"{tid}\tn{tid}\tspecies\t1\t{lin}\n")
    # taxonomy with GCF/GCA regex keys, versionless ids, commas/pipes/space separators
    with open(out / "regex_taxonomy.tsv", "w") as f:
        f.write("GCF\tTaxID\tIdentifiers\n")
        f.write("GCF_000005845.2\t562\tNC_000913.3;NZ_CP178711.1|NZ_CP178708.1,NZ_CP178709.1 NZ_CP178710.1\n")
        f.write("GCF_000006945.2_PRJNA57799\t28901\tNC_003197.2;NC_003277.2\n")
        f.write("GCA_000009045.1\t1423\tNC_000964.3\n")
        f.write("dup\t1280\tNC_000964.3;NZ_CM128240.1\n")  # first row wins for NC_000964.3
        f.write("noTax\t\tNC_002516.2\n")                  # empty TaxID skipped
        f.write("x\t287\tsomething NC_002516.2\n")
        f.write("y\t1639\tfoo|bar\n")


def synth_pafs(out: Path, zymo_paf: Path, seed=7):
    rng = random.Random(seed)
    zl = [l.rstrip("\n").split("\t") for l in open(zymo_paf)]
    targets = sorted({p[5] for p in zl}) + ["NC_000913", "GCF_000005845.2", "gi|123|ref|NC_000964.3|", "NZ_CP178711.1 extra", "unmapped_target", "NC_003277.2.9"]
    lines = []
    for i in range(6000):
        q = f"q{rng.randrange(1500)}"
        qlen = rng.choice([0, 1, 500, 4404, 14963, 100000, 6500183])
        t = rng.choice(targets)
        blen = rng.randrange(0, 2 * max(qlen, 1) + 1)
        row = [q, str(qlen), "0", str(qlen), rng.choice("+-"), t, "5000000", "0", "100", "50", str(blen), "60", "tp:A:P"]
        lines.append("\t".join(row))
    clean = list(lines)
    for t in targets[:12]:  # legacy exact-match shortcut rows (classification.py:52-53,144-151)
        clean.insert(rng.randrange(len(clean)), "\t".join([t, "1000", "0", "1000", "+", t, "1000", "0", "1000", "995", str(rng.choice([989, 990, 1000, 1500])), "60"]))
    (out / "synth_clean.paf").write_text("\n".join(clean) + "\n")
    lines.insert(10, "# comment line")
    lines.insert(20, "short\tline\tonly")
    lines.insert(30, "bad\tNaN\t0\t0\t+\tNC_000913.3\t1\t0\t1\t1\tzz\t0")
    (out / "synth.paf").write_text("\n".join(lines) + "\n")
    # 250k-line stress PAF = zymo x100 with renamed queries (SURVEY.md §6 probe shape)
    big = []
    for k in range(100):
        for p in zl:
            big.append("\t".join([f"{p[0]}_{k}"] + p[1:]))
    (out / "big_zymo_x100.paf").write_text("\n".join(big) + "\n")
    (out / "empty.paf").write_text("")


def run_classifier(mod, paf, tax, hier, tmpdir: Path, procs=2):
    outp = tmpdir / "out.tsv"
    if outp.exists():
        outp.unlink()
    try:
        with contextlib.redirect_stderr(io.StringIO()):
            mod.main_process(str(paf), str(tax), str(hier), str(outp), procs)
    except Exception as e:  # record the failure mode (classification.py raises on empty PAF)
        return {"error": type(e).__name__}
    return {"bytes": outp.read_bytes()}


def make_classify(ref: Path, gdir: Path):
    out = gdir / "classify"
    out.mkdir(parents=True, exist_ok=True)
    shutil.copyfile(ref / "case/truth/zymo_mc/zymo_mc_vs_refs.paf", out / "zymo.paf")
    build_taxonomy_inputs(ref, out)
    synth_pafs(out, out / "zymo.paf")
    cami = load_module(ref / "scripts/classification_cami.py", "ref_classification_cami")
    legacy = load_module(ref / "scripts/classification.py", "ref_classification")
    cases = []
    for paf in ["zymo.paf", "synth.paf", "synth_clean.paf", "big_zymo_x100.paf", "empty.paf"]:
        for tax in ["zymo_taxonomy.tsv", "regex_taxonomy.tsv"]:
            for hier in ["zymo_hierarchy_domain.tsv", "zymo_hierarchy_superkingdom.tsv", "mixed_hierarchy.tsv"]:
                for name, mod in (("cami", cami), ("legacy", legacy)):
                    if paf == "big_zymo_x100.paf" and (tax != "zymo_taxonomy.tsv" or hier == "mixed_hierarchy.tsv"):
                        continue
                    with tempfile.TemporaryDirectory() as td:
                        res = run_classifier(mod, out / paf, out / tax, out / hier, Path(td))
                    key = f"{name}__{paf[:-4]}__{tax[:-4]}__{hier[:-4]}"
                    if "bytes" in res and paf == "big_zymo_x100.paf":
                        import hashlib
                        cases.append({"variant": name, "paf": paf, "taxonomy": tax, "hierarchy": hier,
                                      "sha256": hashlib.sha256(res["bytes"]).hexdigest(), "nbytes": len(res["bytes"])})
                    elif "bytes" in res:
                        (out / f"expect__{key}.tsv").write_bytes(res["bytes"])
                        cases.append({"variant": name, "paf": paf, "taxonomy": tax, "hierarchy": hier, "expect": f"expect__{key}.tsv"})
                    else:
                        cases.append({"variant": name, "paf": paf, "taxonomy": tax, "hierarchy": hier, "error": res["error"]})
    # big file is regenerated deterministically by the tests instead of being committed
    (out / "cases.json").write_text(json.dumps(cases, indent=1))
    print(f"classify: {len(cases)} cases")


def make_limit(ref: Path, gdir: Path):
    out = gdir / "limit"
    out.mkdir(parents=True, exist_ok=True)
    lim = load_module(ref / "scripts/limit_candidates.py", "ref_limit_candidates")
    rng = random.Random(11)
    names = [f"GCF_{rng.randrange(10**9):09d}.{rng.randrange(1, 3)}_ASM{i}v1_genomic.fna.gz" for i in range(400)]
    names += [names[3], names[7]]  # duplicates in the selected list
    names += ["plainname", "GCA_1"]
    # three screen tables, overlapping names, some non-float scores, short lines
    tabs = []
    for t in range(3):
        lines = []
        for n in rng.sample(names, 250):
            sc = rng.choice([f"{rng.random():.6g}", "1", "0.9", "0.95", "nan?", "0.9"])
            lines.append(f"{sc}\t{rng.randrange(1, 1000)}/1000\t{rng.randrange(50)}\t{rng.random():.3g}\t{n}\t[1 seqs] x")
        lines.append("short\tline")
        lines.append("")
        tabs.append(f"score{t}.tab")
        (out / tabs[-1]).write_text("\n".join(lines) + "\n")
    (out / "selected.txt").write_text("\n".join(names) + "\n\n")
    cases = []
    for mx in [1, 5, 120, 5000]:
        for ntab in [0, 1, 3]:
            for dedupe in [False, True]:
                argv = ["--selected", str(out / "selected.txt"), "--output", "OUT", "--max", str(mx), "--assembly-dir", str(out / "no_such_dir")]
                for t in tabs[:ntab]:
                    argv += ["--score-file", str(out / t)]
                if dedupe:
                    argv += ["--dedupe", "--no-download"]
                with tempfile.TemporaryDirectory() as td:
                    o = Path(td) / "limited.txt"
                    a2 = [str(o) if x == "OUT" else x for x in argv]
                    buf = io.StringIO()
                    with contextlib.redirect_stdout(buf):
                        rc = lim.main(a2)
                    key = f"max{mx}_tabs{ntab}_{'dedupe' if dedupe else 'plain'}"
                    (out / f"expect_{key}.txt").write_bytes(o.read_bytes())
                    cases.append({"max": mx, "tabs": tabs[:ntab], "dedupe": dedupe, "rc": rc, "stdout": buf.getvalue(), "expect": f"expect_{key}.txt"})
    (out / "cases.json").write_text(json.dumps(cases, indent=1))
    print(f"limit: {len(cases)} cases")


def make_fallback(ref: Path, gdir: Path):
    """C9: tools/build_id_map.py + tools/mini_classify.py run as scripts on the classify
    fixtures' taxonomy TSVs and PAFs; expected: the id map bytes, the first-hit TSV bytes and
    stdout of each."""
    import subprocess
    out = gdir / "fallback"
    out.mkdir(parents=True, exist_ok=True)
    cdir = gdir / "classify"
    # a PAF whose targets mix versioned / versionless / unknown names and repeated queries
    lines = [l for l in (cdir / "zymo.paf").read_text().splitlines() if l.strip()][:400]
    mixed = []
    for i, l in enumerate(lines):
        p = l.split("\t")
        if i % 7 == 0:
            p[5] = p[5].split(".", 1)[0]          # versionless target
        elif i % 11 == 0:
            p[5] = "NZ_UNKNOWN%d.1" % i           # no TaxID: the next line of that query may hit
        mixed.append("\t".join(p))
    mixed.insert(3, "# comment line")
    mixed.insert(5, "short\tline")
    (out / "mixed.paf").write_text("\n".join(mixed) + "\n")
    cases = []
    for tax in ["zymo_taxonomy.tsv", "regex_taxonomy.tsv"]:
        with tempfile.TemporaryDirectory() as td:
            m = Path(td) / "map.tsv"
            r = subprocess.run([sys.executable, str(ref / "tools/build_id_map.py"), str(cdir / tax), str(m)],
                               capture_output=True, text=True, check=True)
            mkey = f"idmap__{tax[:-4]}.tsv"
            (out / mkey).write_bytes(m.read_bytes())
            for paf, pdir in [("zymo.paf", cdir), ("mixed.paf", out), ("empty.paf", cdir)]:
                o = Path(td) / "fb.tsv"
                r2 = subprocess.run([sys.executable, str(ref / "tools/mini_classify.py"), str(pdir / paf), str(m), str(o)],
                                    capture_output=True, text=True, check=True)
                key = f"mini__{paf[:-4]}__{tax[:-4]}.tsv"
                (out / key).write_bytes(o.read_bytes())
                cases.append({"taxonomy": tax, "paf": paf, "paf_dir": "classify" if pdir == cdir else "fallback",
                              "idmap": mkey, "idmap_stdout": r.stdout.replace(str(m), "MAP"),
                              "expect": key, "stdout": r2.stdout.replace(str(o), "OUT")})
    (out / "cases.json").write_text(json.dumps(cases, indent=1))
    print(f"fallback: {len(cases)} cases")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    ref = Path(a.ref)
    make_classify(ref, HERE)
    make_limit(ref, HERE)
    make_fallback(ref, HERE)
    big = HERE / "classify" / "big_zymo_x100.paf"
    if big.exists():
        big.unlink()  # regenerated by tests from zymo.paf (deterministic), keeps the repo small


if __name__ == "__main__":
    main()
