"""ctypes binding of libivfpq.so (C-ABI declared in include/ivfpq.h).

The library is the only compute path: if it cannot be loaded the import of the
functions that need it fails loudly (there is no CPU fallback).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_PKG)  # chameleon-rag-acceleration_amd/
LIB_PATH = os.environ.get("IVFPQ_LIB") or os.path.join(ROOT, "lib", "libivfpq.so")  # IVFPQ_LIB: A/B builds
CSRC = os.path.join(ROOT, "csrc")

_lock = threading.Lock()
_lib = None

c_f32p = ctypes.POINTER(ctypes.c_float)
c_i64p = ctypes.POINTER(ctypes.c_int64)
c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_handle = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/ivfpq.h one to one, plus the three
# test hooks of include/ivfpq_test.h (used only by tests/).
SIGNATURES = {
    "ivfpq_last_error": (ctypes.c_char_p, []),
    "ivfpq_device_count": (ctypes.c_int, []),
    "ivfpq_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.POINTER(c_handle)]),
    "ivfpq_free": (ctypes.c_int, [c_handle]),
    "ivfpq_train": (ctypes.c_int, [c_handle, ctypes.c_int64, c_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64]),
    "ivfpq_add": (ctypes.c_int, [c_handle, ctypes.c_int64, c_f32p, c_i64p]),
    "ivfpq_precompute_tables_device": (ctypes.c_int, [c_handle, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.POINTER(ctypes.c_uint64)]),
    "ivfpq_search_preassigned_tables_device": (ctypes.c_int, [c_handle, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                              ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "ivfpq_set_inflight": (ctypes.c_int, [c_handle, ctypes.c_int]),
    "ivfpq_get_inflight": (ctypes.c_int, [c_handle]),
    "ivfpq_overlap_built": (ctypes.c_int, []),
    "ivfpq_get_error_count": (ctypes.c_int, [c_handle, c_i64p]),
    "ivfpq_get_repair_stats": (ctypes.c_int, [c_handle, c_i64p, c_i64p]),
    "ivfpq_get_repair_log": (ctypes.c_int, [c_handle, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int)]),
    "ivfpq_set_fault_injection": (ctypes.c_int, [c_handle, ctypes.c_int]),
    "ivfpq_debug_workspace": (ctypes.c_int, [c_handle, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64,
                                             c_i64p]),
    "ivfpq_debug_seed_tau": (ctypes.c_int, [c_handle, ctypes.c_int64, ctypes.c_void_p]),
    "ivfpq_add_device": (ctypes.c_int, [c_handle, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p]),
    "ivfpq_add_preencoded": (ctypes.c_int, [c_handle, ctypes.c_int64, c_i64p, c_u8p, c_i64p]),
    "ivfpq_reset": (ctypes.c_int, [c_handle]),
    "ivfpq_set_nprobe": (ctypes.c_int, [c_handle, ctypes.c_int]),
    "ivfpq_get_nprobe": (ctypes.c_int, [c_handle]),
    "ivfpq_set_list_range": (ctypes.c_int, [c_handle, ctypes.c_int, ctypes.c_int]),
    "ivfpq_search": (ctypes.c_int, [c_handle, ctypes.c_int64, c_f32p, ctypes.c_int, c_f32p, c_i64p]),
    "ivfpq_search_preassigned": (ctypes.c_int, [c_handle, ctypes.c_int64, c_f32p, ctypes.c_int, c_i64p, c_f32p,
                                                c_f32p, c_i64p]),
    "ivfpq_search_device": (ctypes.c_int, [c_handle, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    "ivfpq_search_preassigned_device": (ctypes.c_int, [c_handle, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                       ctypes.c_void_p, ctypes.c_void_p]),
    "ivfpq_serve_request": (ctypes.c_int, [c_handle, c_u8p, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_int, c_u8p, ctypes.c_int64, c_i64p]),
    "ivfpq_coarse_device": (ctypes.c_int, [c_handle, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    "ivfpq_coarse_tables_device": (ctypes.c_int, [c_handle, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                                  ctypes.POINTER(ctypes.c_uint64)]),
    "ivfpq_merge_topk_device": (ctypes.c_int, [ctypes.c_int, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p]),
    "ivfpq_linear_transform_device": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_void_p]),
    "ivfpq_set_timing": (ctypes.c_int, [c_handle, ctypes.c_int]),
    "ivfpq_get_timing": (ctypes.c_int, [c_handle, ctypes.POINTER(ctypes.c_double), c_i64p]),
    "ivfpq_ntotal": (ctypes.c_int64, [c_handle]),
    "ivfpq_is_trained": (ctypes.c_int, [c_handle]),
    "ivfpq_get_dims": (ctypes.c_int, [c_handle] + [ctypes.POINTER(ctypes.c_int)] * 5),
    "ivfpq_get_centroids": (ctypes.c_int, [c_handle, c_f32p]),
    "ivfpq_get_codebook": (ctypes.c_int, [c_handle, c_f32p]),
    "ivfpq_set_trained": (ctypes.c_int, [c_handle, c_f32p, c_f32p]),
    "ivfpq_get_list_sizes": (ctypes.c_int, [c_handle, c_i64p]),
    "ivfpq_get_list": (ctypes.c_int, [c_handle, ctypes.c_int, c_u8p, c_i64p]),
    "ivfpq_get_precomputed_table": (ctypes.c_int, [c_handle, c_f32p]),
    "ivfpq_save": (ctypes.c_int, [c_handle, ctypes.c_char_p]),
    "ivfpq_load": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(c_handle)]),
    "ivfpq_flat_search": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int64, c_f32p, ctypes.c_int64,
                                         c_f32p, ctypes.c_int, ctypes.c_int, c_f32p, c_i64p]),
}


def kernel_source_sha256() -> str:
    """sha256 of what the GPU kernels are compiled from (the kernel source, its
    headers, the Makefile's flags): the key under which counter measurements of
    the kernels stay valid across builds that change host code only."""
    import hashlib

    h = hashlib.sha256()
    for f in ("ivfpq_kernels.hip", "ivfpq_kernels.h", "ivfpq_diag.h", "Makefile"):
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read() + b"\0")
    return h.hexdigest()


def build(force: bool = False) -> str:
    """Compile libivfpq.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    srcs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp", ".h"))]
    srcs += [os.path.join(os.path.dirname(ROOT), "include", h) for h in ("ivfpq.h", "ivfpq_test.h")]
    stale = not os.path.exists(LIB_PATH) or any(os.path.getmtime(s) > os.path.getmtime(LIB_PATH) for s in srcs)
    if force or stale:
        subprocess.check_call(["make", "-s", "-C", CSRC, "-j4"])
    return LIB_PATH


def _preload_torch_runtime():
    # Share one HIP runtime with PyTorch: torch bundles libamdhip64.so.7 with
    # the same soname, so importing torch first makes our NEEDED entry resolve
    # to the already-loaded runtime (device pointers stay valid across both).
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch absent
        pass


def load():
    """Load (building first if stale in a dev tree) and bind libivfpq.so."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH) and os.path.isdir(CSRC):
            try:
                build()
            except Exception as e:  # pragma: no cover
                raise ImportError(f"libivfpq.so missing and build failed: {e}") from e
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"HIP extension missing: {LIB_PATH} (run __graft_entry__.build())")
        _preload_torch_runtime()
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return _lib


def check(rc: int):
    if rc != 0:
        raise RuntimeError(load().ivfpq_last_error().decode("utf-8", "replace"))
