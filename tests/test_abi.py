"""The C-ABI library loads on the CPU host and exports every symbol include/*.h declares
(no compute calls: there is no GPU here)."""
import ctypes
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def declared_symbols():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        txt = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names.update(re.findall(r"\b(hymet_[a-z0-9_]+)\s*\(", txt))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    from hymet_amd import _lib
    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 10
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_bindings_cover_declared_symbols():
    from hymet_amd import _lib
    assert set(declared_symbols()) == set(_lib.exported_symbols())


def test_error_path_without_gpu():
    from hymet_amd import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    rc = lib.hymet_init(0, ctypes.byref(h))
    if rc != 0:  # no device in the build container: must fail loudly with a message
        assert lib.hymet_last_error()
    else:
        lib.hymet_destroy(h)
    assert lib.hymet_version() >= 1


def test_library_is_built_from_these_sources():
    """The shipped libhymet_gpu.so carries the digest of the sources, headers and compile
    commands it was linked from (hymet_amd/build.py); a stale prebuilt library fails here,
    on the build host and on the GPU box alike."""
    from hymet_amd import build
    assert build.is_current(), "libhymet_gpu.so is stale: run python -m hymet_amd.build"


def test_binding_arity_matches_header():
    """Every ctypes signature in hymet_amd/_lib.py has the parameter count its prototype in
    include/hymet_gpu.h declares (a mismatch would pass garbage through the boundary)."""
    from hymet_amd._lib import _SIGS
    txt = re.sub(r"/\*.*?\*/", "", (ROOT / "include" / "hymet_gpu.h").read_text(), flags=re.S)
    bad = []
    for name, (_, args) in _SIGS.items():
        m = re.search(r"\b" + name + r"\s*\((.*?)\);", txt, re.S)
        assert m, name
        body = m.group(1).strip()
        n = 0 if body in ("", "void") else len(body.split(","))
        if n != len(args):
            bad.append((name, n, len(args)))
    assert not bad, bad
