"""Seeded synthetic stand-ins for the benchmark configurations (BASELINE.json configs;
SURVEY.md §8(d)).  The reference ships none of the data, so every configuration is
generated here: genomes are i.i.d. bases; strains/relatives are substitution mutants (the
model of testdataset/mutationGCF.py:4-18: uniform positions, a different base); contigs are
lognormal-length pieces of a sample strain of each taxon, either strand.

    cami-medium (C4): 12 taxa; 62 candidate genomes per taxon at 0.5-4 % divergence from the
        sampled strain (744 candidates, ~3 Gbp, two -I2g index parts); contigs
        lognormal(ln 4000, 1.0) clipped to [1 kbp, 1 Mbp] until ~1 Gbp; sketch DB = Mash
        sketches of the 744 candidates + random decoy sketches (H ~ 1e8 like sketch1).
    cami-low (C3): 8 taxa, 147 candidates, ~100 Mbp of contigs.
    tiny (C1): 3 taxa, 60 contigs of 5-50 kbp.
    cami-medium-zymo: C4's shape on real sequence composition (SURVEY.md §8(d) "Genomes"):
        the taxon backbones are the shipped Zymo genomes (zymo_backbones), each taken to a
        new species by 5-15 % substitutions; three more taxa are sister species of three of
        them (within-genus similarity); candidates are 0.5-2 % strains of the sampled one.
        Real genomes keep their repeats (rRNA operons, IS elements, tandem and
        low-complexity stretches), which i.i.d. backbones lack.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

import numpy as np

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def random_codes(rng, n, gc=0.5):
    p = [(1 - gc) / 2, gc / 2, gc / 2, (1 - gc) / 2]
    return rng.choice(4, size=n, p=p).astype(np.uint8) if gc != 0.5 else rng.integers(0, 4, n, dtype=np.uint8)


def mutate_codes(rng, codes: np.ndarray, rate: float) -> np.ndarray:
    out = codes.copy()
    k = int(rng.binomial(len(codes), rate))
    if k:
        pos = rng.integers(0, len(codes), k)
        out[pos] = (out[pos] + rng.integers(1, 4, k, dtype=np.uint8)) & 3
    return out


def to_ascii(codes: np.ndarray) -> bytes:
    return ACGT[codes].tobytes()


@dataclass
class Workload:
    name: str
    taxa: List[str]
    ref_names: List[str]
    ref_taxon: List[int]
    ref_strain: List[int]
    refs: List[bytes]
    contig_names: List[str]
    contigs: List[bytes]
    contig_taxon: np.ndarray
    taxids: List[int] = field(default_factory=list)

    @property
    def contig_bases(self):
        return int(sum(len(c) for c in self.contigs))

    @property
    def ref_bases(self):
        return int(sum(len(r) for r in self.refs))

    def taxonomy_tsv(self) -> str:
        """detailed_taxonomy.tsv (GCF, TaxID, Identifiers) as scripts/downloadDB.py:178-207 writes it."""
        lines = ["GCF\tTaxID\tIdentifiers"]
        for i, n in enumerate(self.ref_names):
            acc = n.split("_genomic")[0]
            lines.append(f"{acc}\t{self.taxids[self.ref_taxon[i]] + self.ref_strain[i] + 1}\t{n}")
        return "\n".join(lines) + "\n"

    def hierarchy_tsv(self) -> str:
        """taxonomy_hierarchy.tsv rows (TaxID, Name, Rank, ParentTaxID, Lineage) with NCBI-2025
        style 'domain:' labels (scripts/taxonomy_hierarchy.py:37-61 layout)."""
        lines = ["TaxID\tName\tRank\tParentTaxID\tLineage"]
        for t, tax in enumerate(self.taxa):
            base = self.taxids[t]
            genus = f"Genus{t % 7}"
            lin = (f"domain:Bacteria;phylum:Phylum{t % 3};class:Class{t % 4};order:Order{t % 5};"
                   f"family:Family{t % 6};genus:{genus};species:{tax}")
            lines.append(f"{base}\t{tax}\tspecies\t{base - 1}\t{lin}")
            for s in range(max(self.ref_strain) + 1 if self.ref_strain else 0):
                lines.append(f"{base + s + 1}\t{tax} strain {s}\tstrain\t{base}\t{lin};strain:{tax} str. {s}")
        return "\n".join(lines) + "\n"


_CODE = np.full(256, 255, np.uint8)
for _k, _c in zip(b"ACGTacgt", (0, 1, 2, 3, 0, 1, 2, 3)):
    _CODE[_k] = _c


def to_codes(rng, seq: bytes) -> np.ndarray:
    """ASCII -> 2-bit codes; anything but ACGT (N runs, IUPAC codes) becomes a random base."""
    c = _CODE[np.frombuffer(seq, np.uint8)]
    bad = c == 255
    if bad.any():
        c[bad] = rng.integers(0, 4, int(bad.sum()), dtype=np.uint8)
    return c


def zymo_backbones(rng, genomes, n_taxa, sisters_of=(2, 7, 0), species_div=(0.05, 0.15)):
    """Species backbones from real genomes: genomes = [(species, bytes)], one per species
    (the taxa after them are sister species of genomes[sisters_of[k]]).  Every backbone is
    its genome with U[species_div] substitutions (testdataset/mutationGCF.py:4-18), so taxa
    drawn from one genome differ from each other by roughly twice that."""
    src = [g for _, g in genomes] + [genomes[k][1] for k in sisters_of]
    if len(src) < n_taxa:
        raise ValueError(f"{n_taxa} taxa need {n_taxa} backbone sources, have {len(src)}")
    return [mutate_codes(rng, to_codes(rng, src[t]), float(rng.uniform(*species_div))) for t in range(n_taxa)]


def make_cami(rng, n_taxa=12, per_taxon=62, genome_mbp=(3.0, 5.0), div=(0.005, 0.04), contig_gbp=1.0,
              max_contigs=None, name="cami-medium", contig_rng=None, backbones=None) -> Workload:
    """contig_rng: separate generator for the contigs (per-rank samples of one community).
    per_taxon: candidate genomes per taxon (an int, or one count per taxon).
    backbones: one 2-bit code array per taxon (zymo_backbones) instead of i.i.d. ones."""
    taxa = [f"Species{chr(65 + t)} synthetica" for t in range(n_taxa)]
    per = list(per_taxon) if hasattr(per_taxon, "__len__") else [int(per_taxon)] * n_taxa
    ref_names, ref_taxon, ref_strain, refs = [], [], [], []
    sample = []
    for t in range(n_taxa):
        if backbones is not None:
            backbone = backbones[t]
        else:
            L = int(rng.uniform(*genome_mbp) * 1e6)
            backbone = random_codes(rng, L)
        strain = mutate_codes(rng, backbone, 0.01)          # the organism actually sampled
        sample.append(strain)
        for s in range(per[t]):
            r = float(rng.uniform(*div))
            g = mutate_codes(rng, strain, r)
            acc = f"GCF_{(t * 1000 + s) * 7919 % 999999937:09d}.1"
            ref_names.append(f"{acc}_ASM{t}v{s}_genomic")
            ref_taxon.append(t)
            ref_strain.append(s)
            refs.append(to_ascii(g))
    # contigs: lognormal(ln 4000, 1.0) in [1 kbp, 1 Mbp] until contig_gbp
    rng = contig_rng if contig_rng is not None else rng
    cn, cs, ct = [], [], []
    total, target = 0, int(contig_gbp * 1e9)
    i = 0
    while total < target and (max_contigs is None or i < max_contigs):
        t = int(rng.integers(n_taxa))
        g = sample[t]
        L = int(np.clip(rng.lognormal(np.log(4000), 1.0), 1000, min(1_000_000, len(g) - 1)))
        st = int(rng.integers(0, len(g) - L))
        c = g[st:st + L]
        if rng.random() < 0.5:
            c = (3 - c)[::-1]
        cn.append(f"k141_{i}")
        cs.append(to_ascii(c))
        ct.append(t)
        total += L
        i += 1
    w = Workload(name, taxa, ref_names, ref_taxon, ref_strain, refs, cn, cs, np.array(ct, np.int32))
    w.taxids = [100000 + 1000 * t for t in range(n_taxa)]
    return w


def decoy_sketches(rng, n, s):
    h = rng.integers(0, 2 ** 63, size=(n, s), dtype=np.int64).astype(np.uint64) * np.uint64(2) + np.uint64(1)
    h.sort(axis=1)
    return h
