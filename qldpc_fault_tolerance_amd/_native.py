"""ctypes binding of ``libqldpc_hip.so`` (C ABI in ``include/qldpc_hip.h``).

The product path has no CPU fallback: if the HIP library is missing or no GPU
is visible, every entry point raises :class:`NativeUnavailable` naming the
cause.  Build the library in-tree with ``python -c "import __graft_entry__ as g;
g.build()"`` (or :func:`qldpc_fault_tolerance_amd.build.build_native`).
"""
from __future__ import annotations

import ctypes
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QLDPC_LIB") or os.path.join(PKG_DIR, "libqldpc_hip.so")
HIST_BINS = 1025

# Every symbol include/qldpc_hip.h declares (tests check the .so exports them).
EXPORTED = [
    "qldpc_abi_version", "qldpc_last_error", "qldpc_device_count", "qldpc_graph_create", "qldpc_graph_destroy",
    "qldpc_graph_info", "qldpc_bp_create", "qldpc_bp_destroy", "qldpc_bp_set_channel_probs",
    "qldpc_bp_decode_batch", "qldpc_mc_create", "qldpc_mc_destroy", "qldpc_mc_launch", "qldpc_mc_run",
    "qldpc_bp_geometry", "qldpc_bp_engine", "qldpc_phenl_create", "qldpc_phenl_destroy",
    "qldpc_phenl_trace_len", "qldpc_phenl_launch", "qldpc_bp_degree3_slots", "qldpc_bp_create_soft",
    "qldpc_bp_decode_batch_soft", "qldpc_osd_create", "qldpc_osd_destroy", "qldpc_osd_rank",
    "qldpc_osd_decode_batch", "qldpc_osd_gpu_create", "qldpc_osd_gpu_destroy", "qldpc_osd_gpu_decode", "qldpc_osd_gpu_geometry",
    "qldpc_firstmin_create", "qldpc_firstmin_destroy", "qldpc_firstmin_decode", "qldpc_phenl_set_round_firstmin", "qldpc_phenl_set_final_osd",
    "qldpc_bp_bank_stats", "qldpc_bp_create_hbm", "qldpc_mc_set_osd", "qldpc_comm_unique_id",
    "qldpc_comm_init_rank", "qldpc_comm_init_all", "qldpc_comm_rank", "qldpc_comm_allreduce_counters",
    "qldpc_comm_allreduce_counters_group", "qldpc_comm_destroy", "qldpc_mc_run_sharded", "qldpc_sample_errors",
    "qldpc_stream_sync", "qldpc_bp_kernel_id", "qldpc_build_flags", "qldpc_circ_create", "qldpc_circ_set_final_osd", "qldpc_circ_set_sampler",
    "qldpc_circ_info", "qldpc_circ_launch", "qldpc_circ_sample", "qldpc_circ_destroy",
    "qldpc_shard_range", "qldpc_bp_lds_model", "qldpc_m2s_place_model",
]
BUILD_EXPERIMENTAL = 1  # qldpc_build_flags(): the measured-and-not-kept kernel families are compiled in
COMM_ID_BYTES = 128


class NativeUnavailable(RuntimeError):
    pass


ENOTSUP = -4  # QLDPC_ENOTSUP (include/qldpc_hip.h)


class QldpcError(RuntimeError):
    """A negative return code of the C ABI (``rc``: QLDPC_EINVAL, QLDPC_ENOTSUP, ...)."""

    def __init__(self, msg: str = "", rc: int = 0):
        super().__init__(msg)
        self.rc = rc


class Counters(ctypes.Structure):
    """Mirror of ``qldpc_counters``."""

    _fields_ = [
        ("shots", ctypes.c_int64),
        ("failures", ctypes.c_int64),
        ("sector_decodes", ctypes.c_int64 * 2),
        ("sector_iters", ctypes.c_int64 * 2),
        ("sector_nonconv", ctypes.c_int64 * 2),
        ("sector_fail", ctypes.c_int64 * 2),
        ("iter_hist", (ctypes.c_int64 * HIST_BINS) * 2),
    ]


COUNTER_WORDS = ctypes.sizeof(Counters) // 8

_lib = None

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64
_dbl = ctypes.c_double
_pp = ctypes.POINTER(ctypes.c_void_p)


def _declare(L):
    L.qldpc_abi_version.restype = ctypes.c_int
    L.qldpc_abi_version.argtypes = []
    L.qldpc_last_error.restype = ctypes.c_char_p
    L.qldpc_last_error.argtypes = []
    L.qldpc_device_count.restype = ctypes.c_int
    L.qldpc_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
    L.qldpc_graph_create.restype = ctypes.c_int
    L.qldpc_graph_create.argtypes = [ctypes.c_int, _i32, _i32, _vp, _vp, _pp]
    L.qldpc_graph_destroy.restype = ctypes.c_int
    L.qldpc_graph_destroy.argtypes = [_vp]
    L.qldpc_graph_info.restype = ctypes.c_int
    L.qldpc_graph_info.argtypes = [_vp] + [ctypes.POINTER(_i32)] * 5
    L.qldpc_bp_create.restype = ctypes.c_int
    L.qldpc_bp_create.argtypes = [_vp, _vp, _i32, _i32, _dbl, _i32, _i32, _i32, _pp]
    L.qldpc_bp_destroy.restype = ctypes.c_int
    L.qldpc_bp_destroy.argtypes = [_vp]
    L.qldpc_bp_set_channel_probs.restype = ctypes.c_int
    L.qldpc_bp_set_channel_probs.argtypes = [_vp, _vp]
    L.qldpc_bp_decode_batch.restype = ctypes.c_int
    L.qldpc_bp_decode_batch.argtypes = [_vp, _vp, _vp, _vp, _vp, _i64, _vp]
    L.qldpc_bp_create_hbm.restype = ctypes.c_int
    L.qldpc_bp_create_hbm.argtypes = [_vp, _vp, _i32, _dbl, _i32, _pp]
    L.qldpc_bp_create_soft.restype = ctypes.c_int
    L.qldpc_bp_create_soft.argtypes = [_vp, _vp, _i32, _dbl, _i32, _pp]
    L.qldpc_bp_decode_batch_soft.restype = ctypes.c_int
    L.qldpc_bp_decode_batch_soft.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp]
    L.qldpc_osd_create.restype = ctypes.c_int
    L.qldpc_osd_create.argtypes = [_i32, _i32, _vp, _vp, _vp, _i32, _i32, _pp]
    L.qldpc_osd_destroy.restype = ctypes.c_int
    L.qldpc_osd_destroy.argtypes = [_vp]
    L.qldpc_osd_rank.restype = ctypes.c_int
    L.qldpc_osd_rank.argtypes = [_vp, ctypes.POINTER(_i32)]
    L.qldpc_osd_decode_batch.restype = ctypes.c_int
    L.qldpc_osd_decode_batch.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32]
    L.qldpc_osd_gpu_create.restype = ctypes.c_int
    L.qldpc_osd_gpu_create.argtypes = [_vp, _vp, _i32, _i32, _pp]
    L.qldpc_osd_gpu_destroy.restype = ctypes.c_int
    L.qldpc_osd_gpu_destroy.argtypes = [_vp]
    L.qldpc_osd_gpu_decode.restype = ctypes.c_int
    L.qldpc_osd_gpu_geometry.restype = ctypes.c_int
    L.qldpc_firstmin_create.restype = ctypes.c_int
    L.qldpc_firstmin_create.argtypes = [_vp, _vp, _i32, ctypes.c_double, _i32, _vp]
    L.qldpc_firstmin_destroy.restype = ctypes.c_int
    L.qldpc_firstmin_destroy.argtypes = [_vp]
    L.qldpc_firstmin_decode.restype = ctypes.c_int
    L.qldpc_firstmin_decode.argtypes = [_vp, _vp, _vp, _vp, _i64, _vp]
    L.qldpc_phenl_set_round_firstmin.restype = ctypes.c_int
    L.qldpc_phenl_set_round_firstmin.argtypes = [_vp, _vp, _vp]
    L.qldpc_osd_gpu_geometry.argtypes = [_vp] + [ctypes.POINTER(_i32)] * 4
    L.qldpc_osd_gpu_decode.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp]
    L.qldpc_phenl_set_final_osd.restype = ctypes.c_int
    L.qldpc_phenl_set_final_osd.argtypes = [_vp, _vp, _vp]
    L.qldpc_mc_create.restype = ctypes.c_int
    L.qldpc_mc_create.argtypes = [_vp, _vp, _vp, _vp, _pp]
    L.qldpc_mc_set_osd.restype = ctypes.c_int
    L.qldpc_mc_set_osd.argtypes = [_vp, _vp, _vp]
    L.qldpc_mc_destroy.restype = ctypes.c_int
    L.qldpc_mc_destroy.argtypes = [_vp]
    L.qldpc_mc_launch.restype = ctypes.c_int
    L.qldpc_mc_launch.argtypes = [_vp, _dbl, _dbl, _dbl, _u64, _u64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp,
                                  _i32, _vp]
    L.qldpc_mc_run.restype = ctypes.c_int
    L.qldpc_mc_run.argtypes = [_vp, _dbl, _dbl, _dbl, _u64, _u64, _i64, _i32, ctypes.POINTER(Counters), _vp]
    L.qldpc_bp_geometry.restype = ctypes.c_int
    L.qldpc_bp_geometry.argtypes = [_vp] + [ctypes.POINTER(_i32)] * 4
    L.qldpc_bp_engine.restype = ctypes.c_int
    L.qldpc_bp_engine.argtypes = [_vp, ctypes.POINTER(_i32)]
    L.qldpc_bp_bank_stats.restype = ctypes.c_int
    L.qldpc_bp_bank_stats.argtypes = [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]
    L.qldpc_bp_degree3_slots.restype = ctypes.c_int
    L.qldpc_bp_degree3_slots.argtypes = [_vp, ctypes.POINTER(_i32)]
    L.qldpc_phenl_create.restype = ctypes.c_int
    L.qldpc_phenl_create.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _i32, _i64, _pp]
    L.qldpc_phenl_destroy.restype = ctypes.c_int
    L.qldpc_phenl_destroy.argtypes = [_vp]
    L.qldpc_phenl_trace_len.restype = ctypes.c_int
    L.qldpc_phenl_trace_len.argtypes = [_vp, _i32, ctypes.POINTER(_i64)]
    L.qldpc_phenl_launch.restype = ctypes.c_int
    L.qldpc_phenl_launch.argtypes = [_vp, _dbl, _dbl, _dbl, _dbl, _u64, _u64, _i64, _i32, _i32, _vp, _vp, _vp, _vp,
                                     _vp]
    L.qldpc_comm_unique_id.restype = ctypes.c_int
    L.qldpc_comm_unique_id.argtypes = [_vp]
    L.qldpc_comm_init_rank.restype = ctypes.c_int
    L.qldpc_comm_init_rank.argtypes = [ctypes.c_int, _i32, _i32, _vp, _pp]
    L.qldpc_comm_init_all.restype = ctypes.c_int
    L.qldpc_comm_init_all.argtypes = [_i32, _vp, _pp]
    L.qldpc_comm_rank.restype = ctypes.c_int
    L.qldpc_comm_rank.argtypes = [_vp] + [ctypes.POINTER(_i32)] * 3
    L.qldpc_comm_allreduce_counters.restype = ctypes.c_int
    L.qldpc_comm_allreduce_counters.argtypes = [_vp, _vp, _vp]
    L.qldpc_comm_allreduce_counters_group.restype = ctypes.c_int
    L.qldpc_comm_allreduce_counters_group.argtypes = [_pp, _pp, _pp, _i32]
    L.qldpc_comm_destroy.restype = ctypes.c_int
    L.qldpc_comm_destroy.argtypes = [_vp]
    L.qldpc_mc_run_sharded.restype = ctypes.c_int
    L.qldpc_mc_run_sharded.argtypes = [_pp, _pp, _i32, _dbl, _dbl, _dbl, _u64, _u64, _i64, _i32,
                                       ctypes.POINTER(Counters)]
    L.qldpc_sample_errors.restype = ctypes.c_int
    L.qldpc_sample_errors.argtypes = [_dbl, _dbl, _dbl, _u64, _u64, _i64, _i32, _vp, _vp, _vp]
    L.qldpc_bp_kernel_id.restype = ctypes.c_int
    L.qldpc_bp_kernel_id.argtypes = [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]
    L.qldpc_stream_sync.restype = ctypes.c_int
    L.qldpc_stream_sync.argtypes = [_vp]
    L.qldpc_build_flags.restype = ctypes.c_int
    L.qldpc_build_flags.argtypes = []
    L.qldpc_circ_create.restype = ctypes.c_int
    L.qldpc_circ_create.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _i64, _pp]
    L.qldpc_circ_set_final_osd.restype = ctypes.c_int
    L.qldpc_circ_set_final_osd.argtypes = [_vp, _vp, _vp]
    L.qldpc_circ_set_sampler.restype = ctypes.c_int
    L.qldpc_circ_set_sampler.argtypes = [_vp, ctypes.c_int32]
    L.qldpc_circ_info.restype = ctypes.c_int
    L.qldpc_circ_info.argtypes = [_vp] + [ctypes.POINTER(_i32)] * 3
    L.qldpc_circ_launch.restype = ctypes.c_int
    L.qldpc_circ_launch.argtypes = [_vp, _u64, _u64, _i64, _vp, _vp, _vp, _vp]
    L.qldpc_circ_sample.restype = ctypes.c_int
    L.qldpc_circ_sample.argtypes = [_vp, _u64, _u64, _i64, _vp, _vp]
    L.qldpc_bp_lds_model.restype = ctypes.c_int
    L.qldpc_bp_lds_model.argtypes = [_vp, ctypes.POINTER(_i64)]
    L.qldpc_m2s_place_model.restype = ctypes.c_int
    L.qldpc_m2s_place_model.argtypes = [_vp, ctypes.c_int32, ctypes.POINTER(_i64)]
    L.qldpc_shard_range.restype = ctypes.c_int
    L.qldpc_shard_range.argtypes = [_i64, _i32, _i32, ctypes.POINTER(_i64), ctypes.POINTER(_i64)]
    L.qldpc_circ_destroy.restype = ctypes.c_int
    L.qldpc_circ_destroy.argtypes = [_vp]


def lib():
    """The loaded HIP library (raises NativeUnavailable if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeUnavailable(
                f"{LIB_PATH} not found: build the HIP extension first (__graft_entry__.build()); "
                "the engine has no CPU fallback")
        # One HIP runtime per process: load PyTorch's libamdhip64 first so this
        # library binds to it (same SONAME) and shares its device context,
        # allocations and streams instead of initialising a second runtime.
        import torch  # noqa: F401

        L = ctypes.CDLL(LIB_PATH)
        _declare(L)
        if L.qldpc_abi_version() != 1:
            raise NativeUnavailable("libqldpc_hip.so ABI version mismatch")
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().qldpc_last_error().decode(errors="replace")
        raise QldpcError(f"{what} failed (rc={rc}): {msg}", rc)


def experimental_families() -> bool:
    """True when the library carries the opt-in c2s / m2v / 303 / engine-4 kernels
    (built with ``-DQLDPC_EXPERIMENTAL=1``, e.g. ``tools/build_variant.py``)."""
    return bool(lib().qldpc_build_flags() & BUILD_EXPERIMENTAL)


def device_count() -> int:
    c = ctypes.c_int(0)
    rc = lib().qldpc_device_count(ctypes.byref(c))
    return c.value if rc == 0 else 0


def require_gpu() -> None:
    if device_count() <= 0:
        raise NativeUnavailable("no HIP device visible: the MI355X engine needs a GPU (no CPU fallback)")
