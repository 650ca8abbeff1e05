"""ctypes binding of libhymet_gpu.so (include/hymet_gpu.h).

This is the product's only path to the device: if the library or a gfx950 GPU is missing
every call raises -- there is no CPU fallback (the CPU oracle under oracle/ is test
infrastructure and is never imported here)."""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libhymet_gpu.so")

_c = ctypes
_i64, _u64, _i32, _u32, _vp = _c.c_int64, _c.c_uint64, _c.c_int, _c.c_uint32, _c.c_void_p

# name -> (restype, argtypes)
_SIGS = {
    "hymet_version": (_i32, []),
    "hymet_init": (_i32, [_i32, _c.POINTER(_vp)]),
    "hymet_destroy": (_i32, [_vp]),
    "hymet_last_error": (_c.c_char_p, []),
    "hymet_set_stream": (_i32, [_vp, _vp]),
    "hymet_sync": (_i32, [_vp]),
    "hymet_prof_enable": (_i32, [_vp, _i32]),
    "hymet_prof_reset": (_i32, [_vp]),
    "hymet_prof_query": (_i32, [_vp, _c.c_char_p, _c.POINTER(_c.c_double), _c.POINTER(_i64), _c.POINTER(_c.c_double)]),
    "hymet_prof_names": (_i32, [_vp, _c.c_char_p, _i64]),
    "hymet_scratch_trim": (_i32, [_vp, _c.POINTER(_i64)]),
    "hymet_scratch_cached": (_i32, [_vp, _c.POINTER(_i64)]),
    "hymet_scratch_stats": (_i32, [_vp, _vp]),
    "hymet_scratch_reserve": (_i32, [_vp, _i64]),
    "hymet_set_oom_hook": (_i32, [_vp, _vp]),
    "hymet_copy_to_host": (_i32, [_vp, _vp, _vp, _i64, _i32]),
    "hymet_copy_to_device": (_i32, [_vp, _vp, _vp, _i64, _i32]),
    "hymet_pack": (_i32, [_vp, _vp, _i64, _i32, _vp, _vp]),
    "hymet_fasta_index": (_i32, [_vp, _i64, _i32, _i64, _c.POINTER(_i64), _vp, _vp, _vp, _vp, _vp]),
    "hymet_fasta_names": (_i32, [_vp, _vp, _vp, _i64, _vp, _vp]),
    "hymet_fasta_compact": (_i32, [_vp, _vp, _i64, _i64, _vp, _vp, _vp, _i64, _vp, _i64, _vp]),
    "hymet_name_hash": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp]),
    "hymet_sort_pairs_u64": (_i32, [_vp, _vp, _vp, _i64, _i32, _i32]),
    "hymet_scan_u32": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp]),
    "hymet_msh_open": (_i32, [_c.c_char_p, _c.POINTER(_vp)]),
    "hymet_msh_info_get": (_i32, [_vp, _vp]),
    "hymet_msh_copy": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "hymet_msh_upload": (_i32, [_vp, _vp, _i32, _vp, _vp, _i32]),
    "hymet_msh_upload_range": (_i32, [_vp, _vp, _i32, _vp, _vp, _i32, _i64, _i64]),
    "hymet_msh_text_offsets": (_i32, [_vp, _vp, _vp]),
    "hymet_msh_close": (None, [_vp]),
    "hymet_screen_table_slots": (_i64, [_i64]),
    "hymet_screen_table_build": (_i32, [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _i32]),
    "hymet_screen_count": (_i32, [_vp, _vp, _vp, _i64, _i64, _i64, _i32, _u32, _i32, _c.POINTER(_vp), _c.POINTER(_i64),
                                  _c.POINTER(_vp), _c.POINTER(_i64), _c.POINTER(_vp), _u64, _vp, _i64, _vp, _vp]),
    "hymet_screen_stats": (_i32, [_vp, _vp, _i64, _vp, _vp, _vp, _vp]),
    "hymet_mm_sketch": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp, _vp, _i64, _c.POINTER(_i64)]),
    "hymet_mm_index_build": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _c.POINTER(_vp)]),
    "hymet_mm_index_destroy": (_i32, [_vp]),
    "hymet_mm_index_info": (_i32, [_vp, _c.POINTER(_i32), _c.POINTER(_i32), _c.POINTER(_i32), _c.POINTER(_i64)]),
    "hymet_mm_index_max_occ": (_i32, [_vp, _vp, _c.c_float, _c.POINTER(_i32)]),
    "hymet_mm_index_save": (_i32, [_vp, _vp, _c.c_char_p, _i32, _c.POINTER(_i64)]),
    "hymet_mm_index_load": (_i32, [_vp, _c.c_char_p, _i64, _c.POINTER(_vp), _c.POINTER(_i64)]),
    "hymet_mm_index_export": (_i32, [_vp, _vp, _vp, _vp]),
    "hymet_mm_map": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _c.POINTER(_vp)]),
    "hymet_mm_result_size": (_i32, [_vp, _c.POINTER(_i64)]),
    "hymet_mm_result_copy": (_i32, [_vp, _vp, _vp, _vp]),
    "hymet_mm_result_destroy": (_i32, [_vp]),
    "hymet_paf_acc_create": (_i32, [_vp, _c.POINTER(_vp)]),
    "hymet_paf_acc_reset": (_i32, [_vp]),
    "hymet_paf_acc_destroy": (_i32, [_vp]),
    "hymet_paf_acc_info": (_i32, [_vp, _c.POINTER(_i64), _c.POINTER(_vp), _c.POINTER(_vp), _c.POINTER(_vp),
                                  _c.POINTER(_vp), _c.POINTER(_vp)]),
    "hymet_paf_acc_append": (_i32, [_vp, _vp, _vp, _i64, _i64]),
    "hymet_paf_acc_copy": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "hymet_paf_acc_field": (_i32, [_vp, _vp, _i32, _vp]),
    "hymet_mm_map_acc": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp]),
    "hymet_emit_paf": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _c.POINTER(_i64), _vp]),
    "hymet_acc_ref_counts": (_i32, [_vp, _vp, _vp]),
    "hymet_acc_classify": (_i32, [_vp, _vp, _i32, _i32] + [_vp] * 15 + [_c.POINTER(_i32)]),
    "hymet_emit_tsv": (_i32, [_vp, _i32, _i32] + [_vp] * 14 + [_i64, _c.POINTER(_i64)]),
    "hymet_mm_chain_dp": (_i32, [_vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _i32, _c.c_float, _c.c_float, _vp, _vp]),
    "hymet_lca_ref_counts": (_i32, [_vp, _vp, _i64, _vp]),
    "hymet_lca": (_i32, [_vp, _i32, _i32] + [_vp] * 17),
}

_lib = None
_oom_hook = None   # kept referenced: the library holds the function pointer


def _release_torch_cache(_user):
    """The library's out-of-memory hook (hymet_set_oom_hook): its own scratch cache is already
    dropped, so give back the blocks torch's caching allocator holds unused."""
    try:
        import torch
        torch.cuda.empty_cache()
    except Exception:   # a hook must not raise into C; the library then reports its OOM
        pass


class HymetError(RuntimeError):
    pass


def load():
    """Load the HIP library (build it first with `python -m hymet_amd.build` or
    __graft_entry__.build()).  Raises loudly when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("HYMET_LIB", LIB_PATH)  # a compile-time variant (tools/variants.py) for A/B timing
    if not os.path.exists(path):
        raise HymetError(f"{path} not found: build the HIP extension (python -m hymet_amd.build); "
                         "hymet_amd has no CPU fallback")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    global _oom_hook
    _oom_hook = _c.CFUNCTYPE(None, _vp)(_release_torch_cache)
    lib.hymet_set_oom_hook(_c.cast(_oom_hook, _vp), None)
    _lib = lib
    return lib


def exported_symbols():
    return list(_SIGS)


def check(rc: int, what: str):
    if rc != 0:
        msg = load().hymet_last_error()
        raise HymetError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


class Gpu:
    """One libhymet context bound to a torch CUDA(HIP) device and its current stream."""

    def __init__(self, device: int = 0, stream=None):
        import torch

        if not torch.cuda.is_available():
            raise HymetError("no GPU visible: hymet_amd runs on MI355X (gfx950) only")
        self.torch = torch
        self.device = device
        torch.cuda.set_device(device)
        self.dev = torch.device("cuda", device)
        self.lib = load()
        h = _vp()
        check(self.lib.hymet_init(device, _c.byref(h)), "hymet_init")
        self.ctx = h
        self.stream = stream
        self.children = []
        self.bind_stream(stream)

    def fork(self) -> "Gpu":
        """A second library context on its own HIP stream, for work that runs concurrently
        with this context's (mapping batches on two streams); profiled with its parent."""
        child = Gpu(self.device, stream=self.torch.cuda.Stream(device=self.device))
        self.children.append(child)
        return child

    def bind_stream(self, stream=None):
        s = stream if stream is not None else self.torch.cuda.current_stream(self.device)
        check(self.lib.hymet_set_stream(self.ctx, _vp(s.cuda_stream)), "hymet_set_stream")
        self.bound_stream = s   # the torch stream object the library's kernels run on

    def call(self, name, *args):
        check(getattr(self.lib, name)(self.ctx, *args), name)

    def sync(self):
        check(self.lib.hymet_sync(self.ctx), "hymet_sync")
        for ch in self.children:
            ch.sync()

    def prof(self, on: bool = True):
        check(self.lib.hymet_prof_enable(self.ctx, int(on)), "hymet_prof_enable")
        for ch in self.children:
            ch.prof(on)

    def prof_reset(self):
        check(self.lib.hymet_prof_reset(self.ctx), "hymet_prof_reset")
        for ch in self.children:
            ch.prof_reset()

    def prof_table(self):
        """{kernel name: (total ms, launches, algorithmic bytes)} since the last reset, summed
        over this context and its forks."""
        buf = _c.create_string_buffer(1 << 16)
        check(self.lib.hymet_prof_names(self.ctx, buf, 1 << 16), "hymet_prof_names")
        out = {}
        for name in buf.value.decode().split():
            ms, n, b = _c.c_double(), _i64(), _c.c_double()
            check(self.lib.hymet_prof_query(self.ctx, name.encode(), _c.byref(ms), _c.byref(n), _c.byref(b)), "hymet_prof_query")
            out[name] = (ms.value, n.value, b.value)
        for ch in self.children:
            for name, (ms, n, b) in ch.prof_table().items():
                m0, n0, b0 = out.get(name, (0.0, 0, 0.0))
                out[name] = (m0 + ms, n0 + n, b0 + b)
        return out

    def trim(self) -> int:
        """Return the library's cached kernel scratch to HIP; bytes freed."""
        out = _i64()
        check(self.lib.hymet_scratch_trim(self.ctx, _c.byref(out)), "hymet_scratch_trim")
        return out.value

    def reserve(self, nbytes: int):
        """Warm the library's scratch cache with one block of `nbytes` (hymet_scratch_reserve)."""
        check(self.lib.hymet_scratch_reserve(self.ctx, int(nbytes)), "hymet_scratch_reserve")

    def _alloc(self, fn, n, dtype):
        # The library's scratch cache and torch's pool share the HBM: when torch runs out (after
        # releasing its own unused blocks), the library's cached blocks go back and torch retries.
        # The other direction is the library's OOM hook (_release_torch_cache).
        try:
            return fn(int(n), dtype=dtype, device=self.dev)
        except self.torch.OutOfMemoryError:
            if self.trim() == 0:
                raise
            return fn(int(n), dtype=dtype, device=self.dev)

    def empty(self, n, dtype):
        return self._alloc(self.torch.empty, n, dtype)

    def zeros(self, n, dtype):
        return self._alloc(self.torch.zeros, n, dtype)

    def close(self):
        if self.ctx:
            self.lib.hymet_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ptr(t) -> _vp:
    return _vp(t.data_ptr())
