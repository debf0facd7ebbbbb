"""ctypes binding of libgrace_hip.so (the C ABI declared in include/grace_hip.h).

The library is the only compute path of grace_amd: there is no CPU or eager-PyTorch fallback.
If the shared object is missing (not built) or a tensor is not on the GPU, calls raise.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GRACE_HIP_LIB", os.path.join(_HERE, "lib", "libgrace_hip.so"))

P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
F32 = ctypes.c_float
U64 = ctypes.c_uint64
SZ = ctypes.c_size_t
ST = ctypes.c_int

# name -> (restype, argtypes); every symbol declared in include/grace_hip.h
SIGNATURES = {
    "grace_version": (ctypes.c_int, []),
    "grace_last_error": (ctypes.c_char_p, []),
    "grace_read_status": (ST, [P, P, P]),
    "grace_status_take": (ctypes.c_int32, [P]),
    "grace_topk_status_word": (ST, [P]),
    "grace_topk_fallback_spin_limit": (ctypes.c_int64, [ctypes.c_int64]),
    "grace_topk_stream_probe_workspace_bytes": (SZ, [I64]),
    "grace_topk_stream_probe": (ST, [P, P, P, I64, I32, P, SZ, P]),
    "grace_spacer_alloc": (ST, [SZ, P]),
    "grace_spacer_free": (ST, [P]),
    "grace_timer_enable": (ST, [ctypes.c_int]),
    "grace_timer_collect": (ST, [P, P]),
    "grace_event_create": (ST, [P]),
    "grace_event_destroy": (ST, [P]),
    "grace_topk_arm_main_event": (ST, [P]),
    "grace_stream_wait_event": (ST, [P, P]),
    "grace_axpby": (ST, [P, P, F32, F32, P, I64, P]),
    "grace_sub": (ST, [P, P, P, I64, P]),
    "grace_div_scalar": (ST, [P, F32, P, I64, P]),
    "grace_fill": (ST, [P, F32, I64, P]),
    "grace_hbm_probe_elems": (I64, [I64, I32]),
    "grace_hbm_probe": (ST, [P, P, P, I64, I32, P]),
    "grace_accumulate": (ST, [P, P, I64, I32, P]),
    "grace_sign_encode": (ST, [P, P, I64, P]),
    "grace_sign_decode": (ST, [P, P, P, I64, P]),
    "grace_sign_majority": (ST, [P, I32, P, I64, P]),
    "grace_signum_encode": (ST, [P, P, I32, F32, F32, P, I64, P]),
    "grace_sign_step_w1": (ST, [P, P, P, I64, P]),
    "grace_reduce_workspace_bytes": (SZ, [I64]),
    "grace_abs_mean": (ST, [P, I64, P, P, P]),
    "grace_onebit_encode": (ST, [P, I64, P, P, P, P]),
    "grace_onebit_decode": (ST, [P, P, P, I32, P, I64, P]),
    "grace_topk_workspace_bytes": (SZ, [I64, I64]),
    "grace_topk_compress": (ST, [P, I64, I64, P, P, P, SZ, P]),
    "grace_topk_step_dense": (ST, [P, I64, I64, P, P, P, P, I64, P, SZ, P]),
    "grace_topk_residual_step": (ST, [P, P, I32, F32, F32, I64, I64, P, P, P, P, SZ, P]),
    "grace_topk_carry_size": (I64, [I64, I64]),
    "grace_topk_residual_step_swap": (ST, [P, P, I32, F32, F32, I64, I64, P, P, P, P, I64, I32, P, SZ, P]),
    "grace_topk_residual_step_carry": (ST, [P, P, I32, F32, F32, I64, I64, P, P, P, P, I64, I32, P, I64, P, SZ, P]),
    "grace_topk_segmented_small_max": (I32, []),
    "grace_topk_segmented_chunk": (I64, [I32, I32]),
    "grace_topk_segmented_seg_ws_bytes": (I64, [I64, I64]),
    "grace_topk_segmented_fin_blocks": (I32, [I64, I64]),
    "grace_topk_segmented_step": (ST, [P, P, I32, F32, F32, P, P, P, I32, P, I32, P, P, I64, P, P, P, I64, I64, P, P, P,
                                       P, P, I32, P, SZ, I64, P]),
    "grace_topk_segmented_workspace_bytes": (I64, [P, P, I32]),
    "grace_topk_segmented_carry_len": (I64, [I64]),
    "grace_shard_record_words": (SZ, [I64]),
    "grace_shard_select_workspace_bytes": (SZ, [I32, I64]),
    "grace_shard_select": (ST, [P, I32, I32, I64, P, I64, P, P, I64, I64, P, P, P, SZ, P, P]),
    "grace_shard_clear": (ST, [P, I64, I64, P, I64, P]),
    "grace_dgc_workspace_bytes": (SZ, [I64]),
    "grace_dgc_sample": (ST, [P, I64, P, U64, I64, P, P]),
    "grace_dgc_threshold": (ST, [P, I64, P, I64, ctypes.c_double, P, P]),
    "grace_dgc_write": (ST, [P, I64, P, P, P, P]),
    "grace_dgc_write_capped": (ST, [P, I64, P, P, I64, P]),
    "grace_dgc_mask_update_capped": (ST, [P, I64, P, P, P]),
    "grace_dgc_compensate": (ST, [P, P, P, I32, F32, I64, P]),
    "grace_dgc_mask_update": (ST, [P, P, P, I64, P, P]),
    "grace_dgc_select": (ST, [P, I64, P, I64, ctypes.c_double, P, P]),
    "grace_dgc_step_w1": (ST, [P, P, P, I64, P, P, P]),
    "grace_dgc_sample_comp": (ST, [P, P, P, I32, F32, I64, P, U64, I64, P, P]),
    "grace_dgc_sample_kth_workspace_bytes": (SZ, []),
    "grace_dgc_sample_kth": (ST, [P, I64, I64, P, P, P]),
    "grace_dgc_step_w1_fused_workspace_bytes": (SZ, [I64]),
    "grace_dgc_step_w1_fused": (ST, [P, P, P, I32, F32, I64, P, I64, ctypes.c_double, P, P, P, P, P]),
    "grace_sumsq_workspace_bytes": (SZ, []),
    "grace_sumsq": (ST, [P, I64, P, P, P]),
    "grace_clip_by_sumsq": (ST, [P, P, F32, P, I64, P]),
    "grace_pack_bits": (ST, [P, I64, P, P]),
    "grace_sign_encode_bits": (ST, [P, I64, P, P]),
    "grace_unpack_bits": (ST, [P, I64, P, P]),
    "grace_sign_majority_bits": (ST, [P, I64, I32, I64, P, P]),
    "grace_pack2_bytes": (I64, [I64]),
    "grace_pack2": (ST, [P, I64, P, P]),
    "grace_unpack2": (ST, [P, I64, P, P]),
    "grace_tern_pack": (ST, [P, I64, P, P]),
    "grace_tern_unpack": (ST, [P, I64, P, P]),
    "grace_sparse_decode": (ST, [P, P, I64, P, I64, P]),
    "grace_sparse_decode_i64": (ST, [P, P, I64, P, I64, P]),
    "grace_sparse_aggregate": (ST, [P, P, I64, P, I32, F32, P, P, I64, P]),
    "grace_sparse_aggregate_into": (ST, [P, P, I64, P, I32, F32, P, P, I64, P]),
    "grace_sort_payload_workspace_bytes": (SZ, [I64, I64]),
    "grace_sort_payload": (ST, [P, P, I64, I64, P, P, P, P, SZ, P]),
    "grace_sparse_aggregate_sorted": (ST, [P, P, P, I64, I32, F32, P, I64, P]),
    "grace_qsgd_step_w1": (ST, [P, P, P, I32, I64, I32, I32, P, U64, P, P]),
    "grace_qsgd_seg_max": (I32, []),
    "grace_qsgd_compress": (ST, [P, P, P, I32, I64, I32, I32, I32, P, U64, P, P, P, P]),
    "grace_qsgd_compress_at": (ST, [P, I64, P, P, I32, I64, I32, I32, I32, P, U64, P, P, P, P]),
    "grace_qsgd_decompress": (ST, [P, P, I64, I64, I32, P, P, I32, I64, I32, I32, I32, I32, F32, P, P]),
    "grace_qsgd_decompress_records": (ST, [P, I64, I64, I32, I64, P, P, P, I32, I64, I32, I32, P, P]),
    "grace_qsgd_global_workspace_bytes": (SZ, []),
    "grace_qsgd_global_compress": (ST, [P, I64, I32, P, U64, P, P, P, P, P]),
    "grace_randomk_perm_indices": (ST, [U64, I64, I64, P, P]),
    "grace_widen_i32": (ST, [P, I64, P, P]),
    "grace_threshold_count_fixed": (ST, [P, I64, F32, P, P]),
    "grace_threshold_count_dev": (ST, [P, I64, F32, P, P]),
    "grace_threshold_step_w1": (ST, [P, P, I32, F32, F32, I64, F32, P, P, P]),
    "grace_sparse_sub": (ST, [P, P, I64, P, P]),
    "grace_exchange_record_words": (SZ, [I64]),
    "grace_threshold_write_capped": (ST, [P, I64, P, P, I64, P]),
    "grace_sparse_aggregate_capped": (ST, [P, I64, I64, I32, F32, P, P, I64, P, P]),
    "grace_sparse_sub_capped": (ST, [P, I64, P, P]),
    "grace_threshold_write_i64": (ST, [P, I64, P, P, P, P]),
    "grace_terngrad_unit": (I32, []),
    "grace_terngrad_workspace_bytes": (SZ, [I64]),
    "grace_terngrad_slot_bytes": (I32, []),
    "grace_terngrad_shard_stats": (ST, [P, I64, P, P, I32, I64, I64, P, P]),
    "grace_terngrad_shard_encode": (ST, [P, I64, P, P, I32, I64, I64, P, P, U64, P, P, P]),
    "grace_terngrad_scalars": (ST, [P, P, I32, P, P, P, P]),
    "grace_terngrad_compress": (ST, [P, P, P, I32, I64, P, P, U64, P, P, P, P]),
    "grace_terngrad_step_w1": (ST, [P, P, P, I32, I64, P, P, U64, P, P, P, P]),
    "grace_terngrad_decompress": (ST, [P, P, I64, I64, I32, P, I32, I64, I32, F32, P, P]),
    "grace_terngrad_decompress_records": (ST, [P, I64, I32, P, I32, P, P, I32, I64, P, P]),
    "grace_natural_compress": (ST, [P, I64, P, U64, P, P]),
    "grace_natural_compress_at": (ST, [P, I64, I64, P, U64, P, P]),
    "grace_cnat_compress": (ST, [P, I64, P, I32, U64, P, P]),
    "grace_cnat_compress_at": (ST, [P, I64, I64, P, I32, U64, P, P]),
    "grace_natural_decompress": (ST, [P, I64, I32, I64, I32, I32, F32, P, P]),
    "grace_fp16_compress": (ST, [P, P, I64, P]),
    "grace_fp16_decompress": (ST, [P, P, I64, P]),
    "grace_fp16_decompress_aggregate": (ST, [P, I64, I32, I64, F32, P, P]),
    "grace_cast_step_w1": (ST, [P, I64, I32, U64, P, P]),
    "grace_randomk_indices": (ST, [U64, I64, I64, P, P]),
    "grace_gather": (ST, [P, P, I64, P, P]),
    "grace_randomk_step_w1": (ST, [P, P, I32, F32, F32, I64, P, I64, P, P, P]),
    "grace_randomk_shard_step": (ST, [P, P, I32, F32, F32, I64, I64, P, I64, P, P, P]),
    "grace_randomk_decode": (ST, [P, P, I64, P, I64, P]),
    "grace_randomk_step_w1_dense_workspace_bytes": (SZ, [I64, I64]),
    "grace_randomk_group_bytes": (SZ, [I64, I64]),
    "grace_randomk_step_w1_dense": (ST, [P, P, I32, F32, F32, I64, P, I64, P, P, P, P, SZ, P]),
    "grace_threshold_workspace_bytes": (SZ, [I64]),
    "grace_threshold_count": (ST, [P, I64, F32, P, P]),
    "grace_threshold_recount": (ST, [P, I64, F32, P, P]),
    "grace_threshold_write": (ST, [P, I64, P, P, P, P]),
    "grace_powersgd_p": (ST, [P, I64, I64, P, I32, P, P, P]),
    "grace_powersgd_workspace_bytes": (SZ, [I64, I64, I32]),
    "grace_powersgd_p_draw": (ST, [P, I64, I64, U64, I32, P, P, P]),
    "grace_powersgd_qt": (ST, [P, I64, I64, P, I32, P, P, P]),
    "grace_orthogonalize": (ST, [P, I64, I32, P]),
    "grace_normal_orthogonal": (ST, [P, I64, I32, U64, P]),
    "grace_powersgd_outer": (ST, [P, P, I64, I64, I32, P, P, P, P]),
    "grace_powersgd_w1_ok": (I32, [I64, I64, I32]),
    "grace_powersgd_w1_workspace_bytes": (SZ, [I64, I64]),
    "grace_powersgd_w1_compress": (ST, [P, I64, I64, P, U64, P, P, P, SZ, P, P]),
    "grace_normal_fill": (ST, [P, I64, U64, P]),
}


class GraceNativeError(RuntimeError):
    """A native call failed or the native library is unavailable."""


_lock = threading.Lock()
_lib = None


def load():
    """Load (once) and return the ctypes handle; raises GraceNativeError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise GraceNativeError(
                    f"grace_amd native library not found at {LIB_PATH}; build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


_fns = {}


def call(name, *args):
    fn = _fns.get(name)
    if fn is None:   # first call: resolve once (the per-call CDLL attribute lookup costs host time
        fn = _fns[name] = getattr(load(), name)   # on launch-bound steps such as a 4 MiB sign step)
    st = fn(*args)
    if st != 0:
        msg = load().grace_last_error()
        raise GraceNativeError(f"{name} failed ({st}): {msg.decode() if msg else ''}")
    return st


def fn(name):
    """The resolved ctypes function (for launch-bound callers that check the status themselves)."""
    f = _fns.get(name)
    if f is None:
        f = _fns[name] = getattr(load(), name)
    return f


def check(name, st):
    if st != 0:
        msg = load().grace_last_error()
        raise GraceNativeError(f"{name} failed ({st}): {msg.decode() if msg else ''}")


def query(name, *args):
    return getattr(load(), name)(*args)
