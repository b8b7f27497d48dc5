"""ctypes bindings to the in-tree native libraries.

The HIP library must be loaded *after* ``torch`` so that it binds to the HIP runtime torch has
already mapped (same ``libamdhip64.so.7`` soname): kernels then run on torch's device/streams and
take ``torch.cuda.current_stream().cuda_stream`` as their ``hipStream_t``.

Device kernels fail loudly: if a CUDA tensor reaches an op and ``libtmog_hip.so`` cannot be built
or loaded, :func:`hip` raises instead of silently falling back to a slower path.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch

from . import build

_lock = threading.Lock()
_host = None
_hip = None

P = C.c_void_p
I32 = C.c_int32
I64 = C.c_int64
F32 = C.c_float

_HOST_SIGS = {
    "tmog_tree_finalize_cpu": [I64, I32, P, P, P, P, P, P, I32, P, P, I32, I32, I32, P, P, P, I32, P, P, P, P, P,
                               P, P],
    "tmog_hist_build_cpu": [P, I64, I32, P, I32, P, P, P, P, P, P, P, P, I32, I32, I32, P, P, P, I64, P, I32],
    "tmog_split_find_cpu": [P, I32, P, P, P, P, P, I32, I32, I32, P, I32, P, P, P, P, P, P, P, P, P, I64, I32, I32,
                            I32],
    "tmog_partition_cpu": [P, I32, P, P, I32, P, P, P, P, P, I32, P, P, I32],
    "tmog_forest_predict_cpu": [P, I32, I32, P, P, P, P, P, P, P, I32, P, I32, P],
    "tmog_find_splits_cpu": [P, I64, I32, I32, P, P],
    "tmog_murmur3_batch": [P, P, I64, I32, P],
    "tmog_hash_index_batch": [P, P, I64, I32, I32, P],
    "tmog_col_stats_cpu": [P, P, I64, I32, I64, P],
    "tmog_grow_forest_cpu": [P],
    "tmog_grow_status_cpu": [P, P, I32],
    "tmog_grow_nodes_cpu": [P, I32],
    "tmog_grow_leaf_count_cpu": [P, I32],
    "tmog_grow_copy_cpu": [P, I32, P, P, P, P, P, P, P, P],
    "tmog_grow_free_cpu": [P],
    "tmog_shist_new": [I32, I32, I64],
    "tmog_shist_free": [P],
    "tmog_shist_update": [P, P, P, I64],
    "tmog_shist_flush": [P],
    "tmog_shist_merge": [P, P],
    "tmog_shist_size": [P],
    "tmog_shist_bins": [P, P, P],
    "tmog_shist_sum": [P, C.c_double],
    "tmog_tok_run": [P, P, I64, I32, I32, I32],
    "tmog_tok_sizes": [P, P, P],
    "tmog_tok_copy": [P, P, P, P, P],
    "tmog_tok_free": [P],
    "tmog_clean_ascii_lens": [P, P, I64, P, P, P],
    "tmog_first_ids": [P, P, P, I64, P],
}

_HIP_SIGS = {
    "tmog_hip_hist_build": [P, I32, P, P, I32, P, P, P, P, P, I32, I32, I32, P, P, P, I64, P, I32, P, P, I32, I32, I32, P,
                            P, P, I32, P, I32],
    "tmog_hip_hist_stat_chunk": [I32, I32],
    "tmog_hip_hist_subtract": [P, P, P, P, P, P, I32, I64, I64, I32, I32, P],
    "tmog_hip_split_find": [P, I32, P, P, P, P, P, I32, I32, I32, P, I32, P, P, I32, P, P, P, P, P, P, P, P, I32, P,
                            I64, I32, I32, I32, P, P, P],
    "tmog_hip_fp_merge": [P, I32, I32, I64, I32, P, P, P, P, P, P],
    "tmog_hip_rccl_unique_id": [P, I32],
    "tmog_hip_rccl_comm_init": [P, I32, I32],
    "tmog_hip_rccl_comm_destroy": [P],
    "tmog_hip_partition_fused": [P, I32, P, P, P, I32, P, P, P, P, P, P, P, I32, P, P, I64, P, P, P, P, I32],
    "tmog_hip_leaf_collect": [P, P, I32, P, P, P, P, P],
    "tmog_hip_grow_forest": [P],
    "tmog_hip_grow_resident": [P, P],
    "tmog_hip_resident_cap_nodes": [P],
    "tmog_hip_resident_error": [P, I32],
    "tmog_hip_grow_status": [P, P, I32],
    "tmog_hip_grow_nodes": [P, I32],
    "tmog_hip_grow_leaf_count": [P, I32],
    "tmog_hip_grow_copy": [P, I32, P, P, P, P, P, P, P, P],
    "tmog_hip_grow_free": [P],
    "tmog_hip_zero_segments": [P, P, P, I32, I64, I64, I32, I32, P, I32, P],
    "tmog_hip_grow_timing": [P, I32],
    "tmog_hip_boost_epilogue": [P, P, I64, P, P, P, I64, P, P, P, P, I32, P, I32, I64, I64, I64, P, P, I32],
    "tmog_hip_aupr_counts": [P, I32, I32, P, P],
    "tmog_hip_slot_stream": [I32, P, I32],
    "tmog_hip_lr_blocks_per_cu": [I32],
    "tmog_hip_plan_profile": [P, I32],
    "tmog_hip_masked_colsum": [P, P, P, I32, I64, I64, P, P],
    "tmog_hip_wgram": [P, I64, I32, I64, P, I64, I32, P, I64, I32, P, P],
    "tmog_hip_weighted_colsums": [P, I64, I32, I64, P, I64, I32, P, P],
    "tmog_hip_boost_prologue": [P, P, P, P, I32, P, I32, P, P, P, I64, P, P, I64, P, P, P, C.c_float, I32, P],
    "tmog_hip_owlqn_direction": [P, P, P, P, P, P, I32, I32, I32, I32, P, P, P, P, P],
    "tmog_hip_owlqn_candidate": [P, P, P, P, P, P, I32, I32, P, P, P, P],
    "tmog_hip_poisson_pack": [P, I64, P, I32, P, I32, P, P, P, P],
    "tmog_hip_row_uniform": [P, I64, P, I32, P, P],
    "tmog_hip_lr_objective": [P, I64, I32, P, P, I32, I32, I32, P, P, I32, P, I32, P, P, P, I32, P],
    "tmog_hip_lr_objective_mixed": [P, I64, I32, P, I32, I32, P, P, I32, I32, I32, P, P, I32, P, I32, P, P, P, I32,
                                    P],
    "tmog_hip_lr_epilogue_grad": [P, I64, I32, P, P, P, I32, I32, I32, P, I32, P, I32, P, P, P, I32, P],
    "tmog_hip_forest_predict": [P, I32, I32, P, P, I64, P, P, P, P, P, I32, P, I32, P, P],
    "tmog_hip_forest_predict_multi": [P, I32, I32, P, P, I64, P, P, P, P, P, I32, P, I32, P, P, P, P, P, P],
    "tmog_hip_col_stats": [P, P, I64, I32, I64, P, P],
    "tmog_hip_vectorize_numeric": [P, P, P, I64, I32, P, P, P, P, I64, I32, P],
    "tmog_hip_onehot_pivot": [P, P, P, P, I32, I64, P, I64, P],
    "tmog_hip_quantize": [P, I64, I32, P, I32, I32, I32, F32, P, P],
    "tmog_hip_gram_aug": [P, I64, I32, I64, P, P, I32, P, P],
    "tmog_hip_gram_bf16": [P, I64, I64, I32, P, P],
    "tmog_hip_col_bf16_exact": [P, I64, I32, I64, P, P],
    "tmog_hip_bf16_pack": [P, I64, I64, P, P, P, P, P, P, I64, P],
    "tmog_hip_class_colsum": [P, I64, I32, I64, P, I32, I32, P, P],
    "tmog_hip_logistic_grad": [P, P, P, I64, I32, P],
    "tmog_hip_debug_flags": [I32],
    "tmog_hip_csr_spmm": [P, P, P, I64, P, I32, P, I32, I32, P],
    "tmog_hip_csc_spmm_t": [P, P, P, I64, P, I64, P, I32, I32, P, P, P],
    "tmog_hip_softmax_epilogue": [P, I64, I32, I32, P, P, P, I32, P, I32, P],
    "tmog_hip_colsum": [P, I64, I32, I32, P, P],
    "tmog_hip_mlp_bias_sigmoid": [P, I32, I64, I32, P, P],
    "tmog_hip_mlp_sigmoid_backprop": [P, P, I32, I64, I32, I32, P, P],
    "tmog_hip_gather_rows_cols": [P, P, P, I64, I32, P, P],
    "tmog_hip_hash_tokens": [P, P, I64, P, I32, I32, I32, I32, P, P],
    "tmog_hip_hash_tf_rows": [P, I32, I64, I32, I32, P, I64, I64, P],
    "tmog_hip_hash_feat_bytes": [],
    "tmog_hip_code_count": [P, P, I32, I32, I64, P, P],
    "tmog_hip_bucketize": [P, P, I64, P, I32, I32, I32, I32, P, I64, I64, I32, P, P],
    "tmog_hip_date_unit_circle": [P, P, I64, I32, I32, I32, P, I64, I64, P],
    "tmog_hip_rff_summary": [P, P, P, I64, I32, P, I32, P, P],
    "tmog_hip_rff_hist": [P, P, P, I64, I32, P, P, I32, P, P],
    "tmog_hip_binary_areas": [P, I32, P, I64, I32, P, P, P, P],
    "tmog_hip_lr_bf16_blocks_per_cu": [I32, I32],
    "tmog_hip_mnl_epilogue": [P, I64, I32, I32, P, P, P, I32, P, I32, P, P, P, I32, P],
    "tmog_hip_mnl_bf16": [P, I64, I64, I32, P, P, I32, P, I32, I32, P, P, I32, P, P, P, I32, P],
    "tmog_hip_lr_bf16": [P, I64, I64, I32, P, P, I32, P, I32, P, P, I32, P, I32, P, P, P, I32, P],
    "tmog_hip_csv_fields": [P, P, P, I64, I32, I32, P, P, P],
    "tmog_hip_rowgemm": [P, I64, I64, P, I64, I64, I32, I32, I64, P, I64, I64, P, I64, I64, I32, I64, I64, I32, I32, I32,
                         I32, P],
    "tmog_hip_xtd_chunks": [I64, I32, I32, I32, I32],
    "tmog_hip_xtd": [P, I64, I64, P, I64, I64, I32, I64, I64, I32, I32, I32, I32, P, P, P],
    "tmog_hip_csv_parse_num": [P, P, P, I64, I32, P, P, I32, P, P, P, P],
    "tmog_hip_csv_hash_text": [P, P, P, I64, I32, P, I32, P, P, P],
}


_RESTYPES = {"tmog_tok_run": C.c_void_p, "tmog_tok_sizes": None, "tmog_tok_copy": None, "tmog_tok_free": None, "tmog_hip_grow_timing": None, "tmog_clean_ascii_lens": None, "tmog_first_ids": I64,
             "tmog_tree_finalize_cpu": C.c_int64, "tmog_shist_new": C.c_void_p, "tmog_shist_free": None, "tmog_shist_update": None,
             "tmog_shist_flush": None, "tmog_shist_merge": None, "tmog_shist_bins": None,
             "tmog_shist_size": C.c_int64, "tmog_shist_sum": C.c_double,
             "tmog_hip_split_cand_bytes": C.c_size_t, "tmog_hip_rccl_comm_init": C.c_void_p,
             "tmog_grow_forest_cpu": C.c_void_p, "tmog_hip_grow_forest": C.c_void_p,
             "tmog_grow_nodes_cpu": C.c_int64, "tmog_hip_grow_nodes": C.c_int64,
             "tmog_grow_leaf_count_cpu": C.c_int64, "tmog_hip_grow_leaf_count": C.c_int64,
             "tmog_grow_copy_cpu": None, "tmog_hip_grow_copy": None,
             "tmog_grow_free_cpu": None, "tmog_hip_grow_free": None, "tmog_hip_resident_cap_nodes": C.c_int64}


def _declare(lib, sigs):
    for name, args in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = args
        fn.restype = _RESTYPES.get(name, C.c_int)


def _check_loaded_hash(lib, kind: str) -> None:
    """The mapped library reports the sources it was built from (``build._provenance_source``)."""
    fn = getattr(lib, f"tmog_{kind}_source_hash")
    fn.argtypes = []
    fn.restype = C.c_char_p
    got = fn().decode()
    if got != build.source_hash(kind):
        raise RuntimeError(f"loaded {kind} library reports source hash {got}, the tree has {build.source_hash(kind)}")


def host():
    global _host
    if _host is None:
        with _lock:
            if _host is None:
                path = build.build_host()
                build.verify(path, "host")
                lib = C.CDLL(str(path))
                _declare(lib, _HOST_SIGS)
                _check_loaded_hash(lib, "host")
                _host = lib
    return _host


_pyhost = None


def pyhost():
    """The host library's CPython-API entry points (``csrc/host/utf8_pack.cpp``), through ``ctypes.PyDLL``: the
    GIL stays held during the call."""
    global _pyhost
    if _pyhost is None:
        host()                      # built and loaded first (host() takes _lock itself)
        with _lock:
            if _pyhost is None:
                lib = C.PyDLL(str(build.HOST_SO))
                lib.tmog_utf8_offsets.argtypes = [C.py_object, P]
                lib.tmog_utf8_offsets.restype = C.c_int64
                lib.tmog_utf8_copy.argtypes = [C.py_object, P, P]
                lib.tmog_utf8_copy.restype = C.c_int
                _pyhost = lib
    return _pyhost


def _release_torch_cache():
    """Native out-of-memory handler (called from a grower thread, GIL taken by ctypes)."""
    try:
        torch.cuda.empty_cache()
    except Exception:  # noqa: BLE001 - a handler must not unwind into native code
        pass


_OOM_HANDLER_T = C.CFUNCTYPE(None)
_OOM_HANDLER = _OOM_HANDLER_T(_release_torch_cache)      # module-level: must outlive the library's use of it


def hip():
    global _hip
    if _hip is None:
        with _lock:
            if _hip is None:
                if os.environ.get("TMOG_DISABLE_HIP") == "1":
                    raise RuntimeError("HIP kernels disabled by TMOG_DISABLE_HIP=1 but a device tensor was passed")
                path = build.build_hip()
                build.verify(path, "hip")       # never load a library built from other sources
                torch.cuda.init()
                lib = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
                _declare(lib, _HIP_SIGS)
                _check_loaded_hash(lib, "hip")
                dbg = int(os.environ.get("TMOG_HIST_DEBUG", "0"))
                if dbg:
                    lib.tmog_hip_debug_flags(dbg)
                # one device-memory budget: a native buffer growth that runs out of memory first returns
                # torch's cached-but-unused blocks to the device, then retries (ops/csrc/hip/dev_alloc.hpp)
                lib.tmog_hip_set_oom_handler.argtypes = [_OOM_HANDLER_T]
                lib.tmog_hip_set_oom_handler.restype = None
                lib.tmog_hip_set_oom_handler(_OOM_HANDLER)
                lib.tmog_hip_fail_alloc.argtypes = [C.c_long]
                lib.tmog_hip_fail_alloc.restype = None
                _hip = lib
    return _hip


def hip_loaded() -> bool:
    return _hip is not None


def ptr(t) -> int:
    if t is None:
        return None
    return t.data_ptr()


def stream(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def check(rc: int, name: str):
    if rc != 0:
        raise RuntimeError(f"native kernel {name} failed with code {rc}")
