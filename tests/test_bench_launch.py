"""bench.py's multi-rank contract (the driver runs `bench.py --gpus N` under
torch.distributed.run, or bare): `--gpus N` without a launcher starts N rank processes, the
world size must equal N, and rank 0 prints one JSON line for the whole job.

CPU: the launch and the record sharding in gloo dry mode.  GPU: two ranks sharing one GPU
(gloo staging the collectives through the host) must write the same classified_sequences.tsv
as one rank on the same synthetic workload."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env():
    env = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _json_line(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.timeout(300)
def test_gpus2_launches_two_ranks_dry():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       env=_env(), timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 2 and line["backend"] == "gloo" and line["covers_input_once"]
    assert line["shards"][0][0] == 0 and line["shards"][0][1] == line["shards"][1][0]


@pytest.mark.timeout(120)
def test_world_size_must_match_gpus():
    env = _env()
    env.update(RANK="0", WORLD_SIZE="3", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True, env=env,
                       timeout=110)
    assert r.returncode != 0 and "started 3 rank(s)" in r.stderr


SMALL = ["--taxa", "2", "--per-taxon", "3", "--contig-gbp", "0.004", "--db-hashes", "2e4", "--batch-mbp", "1",
         "--map-streams", "1", "--no-cpu", "--steps", "1", "--warmup", "1"]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_two_ranks_tsv_equals_one_rank(tmp_path):
    one, two = tmp_path / "one.tsv", tmp_path / "two.tsv"
    r1 = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--tsv-out", str(one)] + SMALL, capture_output=True,
                        text=True, env=_env(), timeout=280)
    assert r1.returncode == 0, r1.stderr[-3000:]
    r2 = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--backend", "gloo", "--share-gpu", "--tsv-out", str(two)]
                        + SMALL, capture_output=True, text=True, env=_env(), timeout=280)
    assert r2.returncode == 0, r2.stderr[-3000:]
    l1, l2 = _json_line(r1.stdout), _json_line(r2.stdout)
    assert l1["n_gpus"] == 1 and l2["n_gpus"] == 2 and l2["config"]["backend"] == "gloo"
    assert l1["paf_lines"] == l2["paf_lines"] > 0
    a, b = one.read_bytes(), two.read_bytes()
    assert a.count(b"\r\n") > 10 and a == b
