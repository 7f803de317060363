"""ctypes binding of the C-ABI in include/combblas_hip.h (libcombblas_hip.so, in-tree).

There is no fallback: if the HIP library is missing the import fails loudly, so a GPU run can
never silently take another path.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CBH_LIB=<variant> selects a diagnostic build libcombblas_hip_<variant>.so (combblas_amd/build.py
# --stamps / --variant); default is the product
LIB_PATH = os.path.join(_HERE, f"libcombblas_hip_{os.environ['CBH_LIB']}.so" if os.environ.get("CBH_LIB")
                        else "libcombblas_hip.so")

c_int64_p = ctypes.POINTER(ctypes.c_int64)
c_int32_p = ctypes.POINTER(ctypes.c_int32)


class cbh_dcsc(ctypes.Structure):
    _fields_ = [("m", ctypes.c_int64), ("n", ctypes.c_int64), ("nnz", ctypes.c_int64), ("nzc", ctypes.c_int64),
                ("cp", ctypes.c_void_p), ("jc", ctypes.c_void_p), ("ir", ctypes.c_void_p), ("num", ctypes.c_void_p)]


class cbh_phase_stats(ctypes.Structure):
    _fields_ = [("flops", ctypes.c_int64), ("nnz", ctypes.c_int64), ("phases", ctypes.c_int64),
                ("value_sum", ctypes.c_double), ("digest", ctypes.c_uint64)]


class cbh_kernel_times(ctypes.Structure):
    _fields_ = [("symbolic_ms", ctypes.c_double), ("numeric_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("numeric_launches", ctypes.c_int64)]


class cbh_kernel_stat(ctypes.Structure):
    _fields_ = [("ms", ctypes.c_double), ("launches", ctypes.c_int64), ("alg_bytes", ctypes.c_double)]


K_SYM_LARGE, K_SYM_SMALL, K_NUM_LARGE, K_NUM_SMALL, K_MERGE_SYM, K_MERGE_NUM = range(6)
K_NAMES = ["sym_large", "sym_small", "num_large", "num_small", "merge_sym", "merge_num", "num_dense", "sym_mid",
           "num_mid", "sym_bmp"]

ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)
FREE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p)
# per-phase consumer of cbh_spgemm_phased: (user, phase, slot0, slot1, const cbh_mat* view) -> status
FILL_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                           ctypes.c_void_p)
TAKE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                           ctypes.c_void_p)
PHASE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                            ctypes.c_void_p)

# every exported symbol with its signature (restype, argtypes); tests check the header against it
SIGNATURES = {
    "cbh_version": (ctypes.c_char_p, []),
    "cbh_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_ctx_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "cbh_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "cbh_device_pci_id": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]),
    "cbh_ctx_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "cbh_ctx_alloc": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_ctx_free": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "cbh_ctx_set_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "cbh_ctx_stream": (ctypes.c_void_p, [ctypes.c_void_p]),
    "cbh_ctx_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "cbh_ctx_trim": (ctypes.c_int, [ctypes.c_void_p]),
    "cbh_ctx_release": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "cbh_ctx_take_retries": (ctypes.c_int, [ctypes.c_void_p, c_int64_p]),
    "cbh_ctx_memory": (ctypes.c_int, [ctypes.c_void_p, c_int64_p, c_int64_p, c_int64_p, c_int64_p]),
    "cbh_hash_config": (ctypes.c_int, [c_int64_p, c_int64_p, c_int64_p]),
    "cbh_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "cbh_ctx_set_allocator": (ctypes.c_int, [ctypes.c_void_p, ALLOC_FN, FREE_FN, ctypes.c_void_p]),
    "cbh_ctx_set_phase_budget": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
    "cbh_ctx_set_bitmap_fraction": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_double]),
    "cbh_ctx_set_phase_consumer": (ctypes.c_int, [ctypes.c_void_p, PHASE_FN, ctypes.c_void_p]),
    "cbh_mat_upload": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(cbh_dcsc), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_upload_bytes": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(cbh_dcsc), ctypes.c_int64,
                                            ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_value_bytes": (ctypes.c_int64, [ctypes.c_void_p]),
    "cbh_mat_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                      ctypes.c_int, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_clone": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    # user-semiring plans (the numeric launches are C++/HIP: include/combblas_hip/HipSpGEMMDevice.h)
    "cbh_plan_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_plan_info": (ctypes.c_int, [ctypes.c_void_p, c_int64_p, c_int64_p]),
    "cbh_plan_numeric": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32,
                                        ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]),
    "cbh_plan_finish": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]),
    "cbh_plan_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "cbh_plan_col_nnz": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "cbh_plan_spgemm_slots": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64,
                                             ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_wrap_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(cbh_dcsc), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_info": (ctypes.c_int, [ctypes.c_void_p, c_int64_p, c_int64_p, c_int64_p, c_int64_p, ctypes.POINTER(ctypes.c_int)]),
    "cbh_mat_device_arrays": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_void_p)] * 4),
    "cbh_mat_upload_chunks": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                             ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                             ctypes.c_int64, ctypes.c_int64, FILL_FN, ctypes.c_void_p,
                                             ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_download_chunks": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_int64, TAKE_FN, ctypes.c_void_p]),
    "cbh_gen_planted_partition": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64,
                                                 ctypes.c_double, ctypes.c_double, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_row_slice": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_rebase_cols": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]),
    "cbh_mat_copy_out": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]),
    "cbh_mat_free": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "cbh_spgemm": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                  ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_spgemm_symbolic": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_int64_p, c_int64_p,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    "cbh_merge": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                 ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_spgemm_phased": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint32, ctypes.POINTER(cbh_phase_stats)]),
    "cbh_last_kernel_times": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(cbh_kernel_times)]),
    "cbh_ctx_enable_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "cbh_kernel_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(cbh_kernel_stat)]),
    "cbh_kernel_stats_reset": (ctypes.c_int, [ctypes.c_void_p]),
    "cbh_spgemm_masked": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_transpose": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_checksum": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_uint64)]),
    "cbh_mat_checksum_global": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                                ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                                ctypes.POINTER(ctypes.c_uint64)]),
    "cbh_ewise_mult": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_col_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p]),
    "cbh_col_stats_kept": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    "cbh_kselect_cols": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                        ctypes.c_int64, ctypes.c_void_p]),
    "cbh_kselect_hist": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    "cbh_kselect_pick": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int]),
    "cbh_kselect_value": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]),
    "cbh_prune_columns": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mcl_prune_recovery_select": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double,
                                                     ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
                                                     ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mcl_prune_recovery_select_arena": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double,
                                                           ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
                                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                           ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_col_view": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_col_slice": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_col_concat": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_mat_col_concat_consume": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                  ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_arena_create": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_arena_destroy": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "cbh_arena_concat": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_tuples_to_dcsc": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]),
    "cbh_dcsc_to_tuples": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p]),
    "cbh_rmat_edges": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                      ctypes.c_void_p]),
    "cbh_edges_to_csc": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, c_int64_p]),
}

CBH_OK = 0
ERR_CALLBACK = 4006  # returned by a Python per-phase consumer that raised
ERRORS = {3001: "GRIDMISMATCH", 3002: "DIMMISMATCH", 3005: "MATRIXALIAS", 4001: "HIP error", 4002: "out of memory",
          4003: "invalid argument", 4004: "device consistency check failed", 4005: "no HIP device",
          ERR_CALLBACK: "per-phase consumer raised"}

CBH_KEEP_EMPTY_COLS = 0x2
CBH_MASK_PATTERN = 0x4
CBH_MASK_EXPAND = 0x8
CBH_MASK_DOT = 0x10
CBH_PHASE_CHECKSUM = 0x100
CBH_TUPLES_DROP_LOOPS = 0x1


class CombBLASHipError(RuntimeError):
    def __init__(self, code, msg=""):
        self.code = code
        super().__init__(f"combblas_hip error {code} ({ERRORS.get(code, '?')}): {msg}")


_lib = None


def lib():
    """Loads libcombblas_hip.so once. Raises ImportError when it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `python -m combblas_amd.build` "
                              "(there is no CPU fallback)")
        # torch ships its own HIP runtime (torch/lib/libamdhip64.so): it must be the process's one.
        # Loaded after this library's (/opt/rocm's), torch later finds a device while this
        # library's hipGetDeviceCount finds none (GPU box: cb.rmat before the first Context)
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("CBH_LIB") and not hasattr(L, name):
                continue  # a diagnostic variant built from an older tree: entry points it lacks stay unbound
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc, ctx=None):
    if rc != CBH_OK:
        msg = lib().cbh_last_error(ctx).decode() if ctx else ""
        raise CombBLASHipError(rc, msg)
