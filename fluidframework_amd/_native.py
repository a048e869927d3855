"""ctypes binding of the C-ABI in include/mt_replay.h (libmtreplay.so).

The product path has no CPU fallback: if the HIP library is missing or no GPU is visible,
the calls raise."""
import ctypes
import os

import numpy as np

from .wire import CHECKSUM_DTYPE, OP_DTYPE

HERE = os.path.dirname(os.path.abspath(__file__))
MT_E_INVALID, MT_E_HIP, MT_E_NOMEM, MT_E_NODEVICE, MT_E_OVERFLOW, MT_E_STALE_VIEW = -1, -2, -3, -4, -5, -6
# MT_LIB_PATH: an instrumented build of the same sources (e.g. the -DMT_PROF section timers,
# profiles/tools/sections.py); the product library otherwise
LIB_PATH = os.environ.get("MT_LIB_PATH") or os.path.join(HERE, "libmtreplay.so")


class MtOptions(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("seg_capacity", ctypes.c_int32),
                ("block_capacity", ctypes.c_int32), ("heap_capacity", ctypes.c_int32),
                ("text_capacity", ctypes.c_int32), ("props_capacity", ctypes.c_int32),
                ("delta_log_capacity", ctypes.c_int32), ("lds_seg_capacity", ctypes.c_int32),
                ("page_capacity", ctypes.c_int32), ("page_heap_capacity", ctypes.c_int32),
                ("unsettled_capacity", ctypes.c_int32), ("uid_capacity", ctypes.c_int32),
                ("lds_page_capacity", ctypes.c_int32), ("lds_unsettled_capacity", ctypes.c_int32),
                ("lds_page_heap_capacity", ctypes.c_int32), ("lds_narrow_overlap", ctypes.c_int32),
                ("delta_log_mode", ctypes.c_int32), ("live_client", ctypes.c_int32),
                ("live_group_capacity", ctypes.c_int32), ("paged_slices", ctypes.c_int32),
                ("segment_ordinals", ctypes.c_int32), ("overlap_arena_capacity", ctypes.c_int32)]


class MtSegInfo(ctypes.Structure):
    """mt_seg_info (include/mt_replay.h): one segment's read-out."""
    _fields_ = [("row", ctypes.c_int32), ("uid", ctypes.c_uint32), ("position", ctypes.c_int32),
                ("offset", ctypes.c_int32), ("length", ctypes.c_int32), ("seq", ctypes.c_int32),
                ("client", ctypes.c_int32), ("removed_seq", ctypes.c_int32), ("removed_client", ctypes.c_int32),
                ("marker_ref_type", ctypes.c_int32), ("text_len", ctypes.c_int32),
                ("ordinal_len", ctypes.c_int32), ("ordinal", ctypes.c_uint16 * 16)]


# mt_regen_rec (include/mt_replay.h): one op of regeneratePendingOp
REGEN_DTYPE = np.dtype([("kind", "<i4"), ("pos1", "<i4"), ("pos2", "<i4"), ("local_seq", "<i4"),
                        ("text_off", "<u4"), ("text_len", "<u4"), ("props_off", "<u4"), ("flags", "<u4")])


class MtGenCfg(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint32), ("ops", ctypes.c_int32), ("writers", ctypes.c_int32),
                ("lag", ctypes.c_int32), ("seed_len", ctypes.c_int32), ("text_max", ctypes.c_int32),
                ("n_keys", ctypes.c_int32), ("n_values", ctypes.c_int32),
                ("max_keys_per_op", ctypes.c_int32), ("_pad", ctypes.c_int32),
                ("p_insert", ctypes.c_uint64), ("p_insert_remove", ctypes.c_uint64),
                ("p_newline", ctypes.c_uint64), ("p_len_continue", ctypes.c_uint64),
                ("p_insert_props", ctypes.c_uint64), ("p_null", ctypes.c_uint64)]


# (name, restype, argtypes) for every symbol of include/mt_replay.h
_P, _I, _U32, _U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64
SIGNATURES = [
    ("mt_create", _P, [_U32, _P]),
    ("mt_destroy", None, [_P]),
    ("mt_last_error", ctypes.c_char_p, [_P]),
    ("mt_num_docs", _U32, [_P]),
    ("mt_load_initial_text", _I, [_P, _P, _P]),
    ("mt_start_collaboration", _I, [_P, _P, _P]),
    ("mt_reset", _I, [_P]),
    ("mt_apply_ops", _I, [_P, _P, _P, _U64, _P, _U64, _P, _U64]),
    ("mt_load_snapshots", _I, [_P, _P, _P, _P, _U64, _P, _U64, _P, _U64, _P, _P]),
    ("mt_extract_snapshots", _I, [_P, _P, _P, _P, _P, _P, _P]),
    ("mt_snapshots_upload", _P, [_P, _P, _P, _P, _U64, _P, _U64, _P, _U64, _P, _P]),
    ("mt_snapshots_upload_range", _P, [_P, _U32, _U32, _P, _P, _P, _U64, _P, _U64, _P, _U64, _P, _P]),
    ("mt_snapshots_load_async", _I, [_P, _P]),
    ("mt_snapshots_free", None, [_P]),
    ("mt_batch_upload", _P, [_P, _P, _P, _U64, _P, _U64, _P, _U64]),
    ("mt_batch_apply_async", _I, [_P, _P]),
    ("mt_batch_num_ops", _U64, [_P]),
    ("mt_batch_free", None, [_P]),
    ("mt_host_alloc", ctypes.c_void_p, [ctypes.c_uint64]),
    ("mt_host_free", None, [ctypes.c_void_p]),
    ("mt_sync", _I, [_P]),
    ("mt_last_kernel_ms", ctypes.c_float, [_P]),
    ("mt_set_stream_priority", ctypes.c_int, [_P, ctypes.c_int]),
    ("mt_last_load_ms", ctypes.c_float, [_P]),
    ("mt_last_hbm_docs", _I, [_P, _P]),
    ("mt_last_paged_peaks", _I, [_P, _P]),
    ("mt_last_grown", _I, [_P, _P]),
    ("mt_generate", _P, [_P, _P, _U32, _P]),
    ("mt_generate_docs", _P, [_P, _P, _U32, _P, _P, _P]),
    ("mt_generated_seeds_docs", _I, [_P, _P, _U32, _P, _P, _P]),
    ("mt_generated_seeds", _I, [_P, _P, _U32, _P, _P]),
    ("mt_batch_sizes", _I, [_P, _P, _P, _P]),
    ("mt_batch_download", _I, [_P, _P, _P, _P, _P]),
    ("mt_get_status", _I, [_P, _P]),
    ("mt_get_length", _I, [_P, _U32, _P]),
    ("mt_get_text", _I, [_P, _U32, _P, _U32, _P]),
    ("mt_get_prop_runs", _I, [_P, _U32, _P, _U32, _P, _P, _U32, _P]),
    ("mt_get_segments", _I, [_P, _U32, _P, _U32, _P, _P, _U32, _P]),
    ("mt_get_segment_props", _I, [_P, _U32, _U32, _P, _U32, _P]),
    ("mt_get_all_segment_props", _I, [_P, _U32, _P, ctypes.c_uint64, _P]),
    ("mt_get_overlap_arena", _I, [_P, _U32, _P]),
    ("mt_get_delta_log", _I, [_P, _U32, _P, _U32, _P]),
    ("mt_delta_log_reset", _I, [_P]),
    ("mt_debug_raw", _I, [_P, _U32, _P, _U32, _P, _P]),
    ("mt_debug_prof", _I, [_P, _P, _I]),
    ("mt_maintenance_counts", _I, [_P, _P]),
    ("mt_checksums", _I, [_P, _P]),
    ("mt_checksums_device", _I, [_P, _P]),
    ("mt_regenerate_pending", _I, [_P, _U32, _P, _U32, _P, _P, _U32, _P, _U32]),
    ("mt_pending_counts", _I, [_P, _P]),
    ("mt_debug_heap", _I, [_P, _U32, _P, _U32, _P, _P, _U32, _P]),
    ("mt_get_containing_segment", _I, [_P, _U32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P, _U32]),
    ("mt_get_segment_by_uid", _I, [_P, _U32, _U32, ctypes.c_int32, ctypes.c_int32, _P, _P, _U32]),
    ("mt_get_view_lengths", _I, [_P, _U32, _P, _P, _P, _P]),
]

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"HIP replay library missing: {LIB_PATH} (run __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        if os.environ.get("MT_LIB_PATH") and not hasattr(lib, name):
            continue   # an older variant build (A/B runs) lacks later entry points
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def gen_cfg(cfg):
    from .wire import gen_thresholds
    return MtGenCfg(seed=cfg["seed"], ops=cfg["ops"], writers=cfg["writers"], lag=cfg["lag"],
                    seed_len=cfg["seed_len"], text_max=cfg["text_max"], n_keys=cfg["n_keys"],
                    n_values=cfg["n_values"], max_keys_per_op=cfg["max_keys_per_op"],
                    **gen_thresholds(cfg))
