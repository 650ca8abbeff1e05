"""Build libhymet_gpu.so in-tree (hipcc, gfx950 only).  Called by __graft_entry__.build()."""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libhymet_gpu.so")
OBJ = os.path.join(HERE, "csrc", "build")

FLAGS = ["-O3", "--offload-arch=gfx950", "-fPIC", "-std=c++17", "-ffp-contract=off",
         "-Wall", "-Wno-unused-function", "-Wno-unused-result", "-I", os.path.join(HERE, "..", "include")]


def _needs(obj, src, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in [src] + deps)


def build(verbose=False, jobs=8, extra=(), out=OUT, obj=OBJ):
    """extra / out / obj: compile-time variants for A/B timing (tools/variants.py)."""
    os.makedirs(obj, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    deps = glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(HERE, "..", "include", "*.h"))
    objs, procs = [], []
    for s in srcs:
        o = os.path.join(obj, os.path.basename(s) + ".o")
        objs.append(o)
        if _needs(o, s, deps):
            cmd = ["hipcc", *FLAGS, *extra, "-c", s, "-o", o]
            if verbose:
                print(" ".join(cmd))
            procs.append((s, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
            while len([p for _, p in procs if p.poll() is None]) >= jobs:
                procs[0][1].wait()
    for s, p in procs:
        log = p.communicate()[0].decode()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed on {s}:\n{log}")
        if log.strip() and verbose:
            print(log)
    if not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        cmd = ["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs]
        subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
