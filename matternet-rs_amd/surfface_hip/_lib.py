"""Loader for libmatternet_hip.so (the C ABI in include/matternet_hip.h).

The product path has no CPU fallback: if the HIP library is missing or fails
to load, every op raises.  Build it with `make -C matternet-rs_amd/csrc` (or
`python -c "import __graft_entry__ as g; g.build()"`).
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(PKG_DIR), "libmatternet_hip.so")
# The tuning build (-DMN_TUNING: reads the MN_* A/B knobs, carries the timing
# probes) for scripts/ and the tests of alternative generator paths; the
# release library above ignores every MN_* tuning variable.
TUNING_LIB_PATH = os.path.join(os.path.dirname(PKG_DIR), "libmatternet_hip_tuning.so")

MN_OK, MN_EINVAL, MN_ENOMEM, MN_ENONFINITE, MN_ECAP, MN_EHIP, MN_ENOTSUP, MN_ECOMM = \
    0, -1, -2, -3, -4, -5, -6, -7
_NAMES = {-1: "MN_EINVAL", -2: "MN_ENOMEM", -3: "MN_ENONFINITE", -4: "MN_ECAP", -5: "MN_EHIP",
          -6: "MN_ENOTSUP", -7: "MN_ECOMM"}

MN_L2SQ, MN_COS_RECT, MN_L2 = 0, 1, 2


class MnError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_NAMES.get(code, code)}: {msg}")
        self.code = code


class KnnOpts(C.Structure):
    _fields_ = [("k", C.c_int32), ("metric", C.c_int32), ("exclude_self", C.c_int32),
                ("margin", C.c_int32), ("timing", C.c_int32), ("algo", C.c_int32),
                ("stream", C.c_void_p)]


# enum mn_knn_algo: candidate generator of mn_knn_f32 (outputs are identical)
MN_KNN_AUTO, MN_KNN_F32, MN_KNN_BF16X3, MN_KNN_BF16X1 = 0, 1, 2, 3


class KnnStats(C.Structure):
    _fields_ = [("n_queries", C.c_int64), ("n_uncertified", C.c_int64), ("slices", C.c_int32),
                ("list_len", C.c_int32), ("ms_norms", C.c_float), ("ms_gram", C.c_float),
                ("ms_rerank", C.c_float), ("ms_fallback", C.c_float), ("ms_total", C.c_float),
                ("algo", C.c_int32), ("ms_sample", C.c_float), ("ms_sweep", C.c_float),
                ("sample_rows", C.c_int64), ("n_candidates", C.c_int64),
                ("sweep_slices", C.c_int32), ("sweep_cap", C.c_int32),
                ("n_escalated", C.c_int64), ("ms_escalate", C.c_float), ("n_root_rescan", C.c_int32)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


MN_F32, MN_F64 = 0, 1
MN_W_GIVEN, MN_W_RATIONAL = 0, 1
MN_SYM_UNION, MN_SYM_MAX = 0, 1


class LapOpts(C.Structure):
    _fields_ = [("weight_kernel", C.c_int32), ("symmetrise", C.c_int32), ("normalize", C.c_int32),
                ("reserved0", C.c_int32), ("eps", C.c_double), ("sigma", C.c_double),
                ("p", C.c_double), ("weight_threshold", C.c_double), ("stream", C.c_void_p)]


class Csr(C.Structure):
    _fields_ = [("n_rows", C.c_int64), ("n_cols", C.c_int64), ("nnz", C.c_int64),
                ("indptr", C.c_void_p), ("indices", C.c_void_p), ("values", C.c_void_p),
                ("value_type", C.c_int32), ("caller_owned", C.c_int32)]


class LapStats(C.Structure):
    _fields_ = [("nnz", C.c_int64), ("big_rows", C.c_int64), ("hub_rows", C.c_int64),
                ("ms_total", C.c_float), ("reserved0", C.c_float)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_ if f != "reserved0"}


class CosOpts(C.Structure):
    _fields_ = [("topk", C.c_int32), ("margin", C.c_int32), ("eps", C.c_double),
                ("sigma", C.c_double), ("p", C.c_double), ("timing", C.c_int32),
                ("reserved0", C.c_int32), ("stream", C.c_void_p)]


MN_G_TAUMODE, MN_G_ENERGYMAPS, MN_G_SPECTRAL = 0, 1, 2
MN_TAU_FIXED, MN_TAU_MEDIAN, MN_TAU_MEAN, MN_TAU_PERCENTILE = 0, 1, 2, 3


class EnergyOpts(C.Structure):
    _fields_ = [("g_mode", C.c_int32), ("tau_mode", C.c_int32), ("tau_param", C.c_double),
                ("timing", C.c_int32), ("reserved0", C.c_int32), ("stream", C.c_void_p)]


class EnergyStats(C.Structure):
    _fields_ = [("entries", C.c_int64), ("symmetric", C.c_int32), ("reserved0", C.c_int32),
                ("ms_rows", C.c_float), ("ms_total", C.c_float)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_ if f != "reserved0"}


P = C.c_void_p
I64 = C.c_int64
I32 = C.c_int32

# name -> (restype, argtypes); every symbol declared in include/matternet_hip.h
SIGNATURES = {
    "mn_version": (C.c_int, []),
    "mn_last_error": (C.c_char_p, []),
    "mn_device_alloc": (C.c_int, [C.c_size_t, C.POINTER(C.c_void_p)]),
    "mn_device_free": (C.c_int, [P]),
    "mn_memcpy_h2d": (C.c_int, [P, P, C.c_size_t, P]),
    "mn_memcpy_d2h": (C.c_int, [P, P, C.c_size_t, P]),
    "mn_memcpy_d2d": (C.c_int, [P, P, C.c_size_t, P]),
    "mn_stream_synchronize": (C.c_int, [P]),
    "mn_fill_uniform_f32": (C.c_int, [P, I64, I32, C.c_uint64, I64, P]),
    "mn_libm_f32": (C.c_int, [P, I64, C.c_uint32, I32, P, P]),
    "mn_knn_f32": (C.c_int, [P, I64, I32, C.POINTER(KnnOpts), P, P]),
    "mn_knn_f32_qc": (C.c_int, [P, I64, P, I64, I32, I64, I64, C.POINTER(KnnOpts), P, P]),
    "mn_knn_merge_f32": (C.c_int, [P, P, I32, I64, I32, P, P, P]),
    "mn_knn_l2_f64": (C.c_int, [P, I64, P, I64, I32, I32, P, I32, I32, P, P, P]),
    "mn_libm_pow_f64": (C.c_int, [P, P, I64, P, P]),
    "mn_knn_sharded_f32": (C.c_int, [P, I64, I32, P, C.POINTER(KnnOpts), I64, P, P]),
    "mn_knn_sharded_sim_f32": (C.c_int, [P, I64, I32, I32, C.POINTER(KnnOpts), P, P, P]),
    "mn_knn_sharded_threads_f32": (C.c_int, [P, I64, I32, I32, C.POINTER(KnnOpts), P, P, P]),
    "mn_shard_quiesce": (C.c_int, [C.c_double]),
    "mn_sym_share_table": (C.c_int, [I32, I32, I32, P, I64, P]),
    "mn_rccl_unique_id": (C.c_int, [P]),
    "mn_rccl_comm_init": (C.c_int, [P, I32, I32, C.POINTER(C.c_void_p)]),
    "mn_rccl_comm_destroy": (C.c_int, [P]),
    "mn_rccl_set_timeout": (C.c_int, [C.c_double]),
    "mn_knn_last_stats": (C.c_int, [C.POINTER(KnnStats)]),
    "mn_laplacian_from_knn": (C.c_int, [P, P, I32, I64, I32, C.POINTER(LapOpts), C.POINTER(Csr), P]),
    "mn_csr_free": (C.c_int, [C.POINTER(Csr)]),
    "mn_lap_last_stats": (C.c_int, [C.POINTER(LapStats)]),
    "mn_energy_rows": (C.c_int, [C.POINTER(Csr), P, I64, I32, C.POINTER(EnergyOpts), P, P, P]),
    "mn_diffuse_rows": (C.c_int, [C.POINTER(Csr), P, I32, I64, I32, C.c_double, I32, P, P]),
    "mn_energy_signals": (C.c_int, [C.POINTER(Csr), P, I64, I32, I32, P, P, P]),
    "mn_bc_knn_f32": (C.c_int, [P, P, I64, I32, I32, C.c_float, C.c_float, P, P, P]),
    "mn_nearest_centroid_f32": (C.c_int, [P, I64, P, I64, I32, P, P, P]),
    "mn_mst_candidate_graph_f32": (C.c_int, [P, P, I64, I32, I32, I32, I32, P, P, P, P, P, P]),
    "mn_laplacian_matvec_rows": (C.c_int, [C.POINTER(Csr), P, I32, I64, I32, P, P]),
    "mn_normalise_lambdas": (C.c_int, [P, I64, P, P]),
    "mn_energy_last_stats": (C.c_int, [C.POINTER(EnergyStats)]),
    "mn_sorted_index": (C.c_int, [P, I64, P, P, P, P]),
    "mn_sorted_range_bylambda": (C.c_int, [P, P, I64, C.c_double, P, I64, C.c_int32, C.c_double,
                                           P, P, P, P]),
    "mn_sorted_k_nearest_by_lambda": (C.c_int, [P, P, I64, C.c_double, P, I64, C.c_int32,
                                                C.c_double, C.c_int32, C.c_double, C.c_double,
                                                C.c_double, P, P, P, P]),
    "mn_sparsify_rows": (C.c_int, [P, P, I64, I32, C.c_double, I32, P, P, P, P, P]),
    "mn_sparsify_sfgrass": (C.c_int, [C.POINTER(Csr), I64, C.c_double, C.POINTER(Csr), P, P]),
    "mn_knn_cos_columns_f32": (C.c_int, [P, I64, I32, C.POINTER(CosOpts), P, P, P]),
    "mn_knn_cos_columns_f64": (C.c_int, [P, I64, I32, C.POINTER(CosOpts), P, P, P]),
    "mn_standardize_columns_f64": (C.c_int, [P, I64, I32, P, P]),
    "mn_cos_last_stats": (C.c_int, [C.POINTER(KnnStats)]),
    "mn_knn_cos_bf16": (C.c_int, [P, I64, I32, C.POINTER(CosOpts), P, P, P]),
    "mn_knn_cos_bf16_qc": (C.c_int, [P, I64, P, I64, I32, I64, I64, C.POINTER(CosOpts), P, P, P]),
    "mn_bf16_last_stats": (C.c_int, [C.POINTER(KnnStats)]),
    "mn_search_lambda_aware": (C.c_int, [P, I32, I64, I32, P, P, P, I64, I32, C.c_double, P,
                                         P, P]),
    "mn_search_lambda_aware_hybrid": (C.c_int, [P, I32, I64, I32, P, P, P, I64, I32,
                                                C.c_double, P, P, P]),
}
MN_SPARSIFY_SFGRASS, MN_SPARSIFY_INLINE = 0, 1

_LIB = None
_LOADED = {}


def _load(path: str) -> C.CDLL:
    if path not in _LOADED:
        if not os.path.exists(path):
            raise ImportError(f"{os.path.basename(path)} not built at {path}; "
                              "run `make -C matternet-rs_amd/csrc`")
        L = C.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LOADED[path] = L
    return _LOADED[path]


def lib() -> C.CDLL:
    """Load the HIP library (raises loudly if it is missing: no fallback path)."""
    global _LIB
    if _LIB is None:
        _LIB = _load(LIB_PATH)
    return _LIB


def select_tuning_library() -> None:
    """Scripts: make every op of this process use the tuning build (MN_* knobs
    and timing probes honoured).  Call before the first op."""
    global _LIB
    _LIB = _load(TUNING_LIB_PATH)


@contextlib.contextmanager
def use_tuning():
    """Tests of alternative paths: the ops inside the block run on the tuning
    build (same sources, MN_* knobs honoured); the release library after."""
    global _LIB
    prev = lib()
    _LIB = _load(TUNING_LIB_PATH)
    try:
        yield _LIB
    finally:
        _LIB = prev


def check(rc: int) -> None:
    if rc != MN_OK:
        msg = lib().mn_last_error()
        raise MnError(rc, msg.decode() if msg else "")
