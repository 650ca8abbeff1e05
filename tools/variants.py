"""Build compile-time variants of libhymet_gpu.so for A/B timing on the GPU box:

    python tools/variants.py NAME -DMACRO=V ...   ->  tools/var/NAME/libhymet_gpu.so
    HYMET_LIB=tools/var/NAME/libhymet_gpu.so python bench.py ...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hymet_amd import build  # noqa: E402

if __name__ == "__main__":
    name, flags = sys.argv[1], sys.argv[2:]
    d = os.path.join(ROOT, "tools", "var", name)
    print(build.build(extra=flags, out=os.path.join(d, "libhymet_gpu.so"), obj=os.path.join(d, "obj")))
