"""Build libhymet_gpu.so in-tree (hipcc, gfx950 only).  Called by __graft_entry__.build().

Rebuild decisions are content-addressed: every object carries a `.sig` file holding the
sha256 of its source, every header it may include and the exact compile command, and the
library carries the digest of its objects' signatures.  A changed flag, a copied tree with
shuffled mtimes or a stale prebuilt object therefore always triggers a rebuild."""
import glob
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libhymet_gpu.so")
OBJ = os.path.join(HERE, "csrc", "build")

FLAGS = ["-O3", "--offload-arch=gfx950", "-fPIC", "-std=c++17", "-ffp-contract=off",
         "-Wall", "-Wno-unused-function", "-Wno-unused-result", "-I", os.path.join(HERE, "..", "include")]
LINK = ["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC"]


def _digest(paths, cmd) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    h.update("\0".join(cmd).encode())
    return h.hexdigest()


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def build(verbose=False, jobs=8, extra=(), out=OUT, obj=OBJ):
    """extra / out / obj: compile-time variants for A/B timing (tools/variants.py)."""
    os.makedirs(obj, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    deps = sorted(glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(HERE, "..", "include", "*.h")))
    objs, sigs, procs = [], [], []
    for s in srcs:
        o = os.path.join(obj, os.path.basename(s) + ".o")
        cmd = ["hipcc", *FLAGS, *extra, "-c", s, "-o", o]
        sig = _digest([s] + deps, cmd)
        objs.append(o)
        sigs.append(sig)
        if not os.path.exists(o) or _read(o + ".sig") != sig:
            if verbose:
                print(" ".join(cmd))
            if os.path.exists(o + ".sig"):
                os.unlink(o + ".sig")
            procs.append((s, o, sig, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
            while len([p for *_, p in procs if p.poll() is None]) >= jobs:
                next(p for *_, p in procs if p.poll() is None).wait()
    for s, o, sig, p in procs:
        log = p.communicate()[0].decode()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed on {s}:\n{log}")
        if log.strip() and verbose:
            print(log)
        with open(o + ".sig", "w") as f:
            f.write(sig + "\n")
    lib_sig = hashlib.sha256(("\n".join(sigs) + "\0" + " ".join(LINK)).encode()).hexdigest()
    # relink whenever an object was just compiled: the library's signature file alone is not
    # trusted in place of the binary (a shipped .so with a matching .sig beside freshly
    # compiled objects is relinked from those objects)
    if procs or not os.path.exists(out) or _read(out + ".sig") != lib_sig:
        subprocess.check_call([*LINK, "-o", out, *objs])
        with open(out + ".sig", "w") as f:
            f.write(lib_sig + "\n")
    return out


def is_current(out=OUT, obj=OBJ) -> bool:
    """True when the library on disk was linked from objects of the present sources."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    deps = sorted(glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(HERE, "..", "include", "*.h")))
    sigs = [_digest([s] + deps, ["hipcc", *FLAGS, "-c", s, "-o", os.path.join(obj, os.path.basename(s) + ".o")])
            for s in srcs]
    return _read(out + ".sig") == hashlib.sha256(("\n".join(sigs) + "\0" + " ".join(LINK)).encode()).hexdigest()


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
