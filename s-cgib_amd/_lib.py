"""ctypes binding of libscgib.so (the C-ABI declared in include/scgib.h).

There is no fallback: if the library is missing or cannot be loaded, every
op raises.  Build it with ``__graft_entry__.build()`` or
``make -C s-cgib_amd/csrc``.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# SCGIB_LIB: debug builds only (tools/phase_trace.py loads libscgib_trace.so)
LIB_PATH = os.environ.get("SCGIB_LIB") or os.path.join(HERE, "libscgib.so")

_P, _I64, _I32, _F, _D = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float, ctypes.c_double

# name -> (restype, argtypes); mirrors include/scgib.h exactly
SIGNATURES = {
    "scgib_abi_version": (ctypes.c_int, []),
    "scgib_set_recon_fold": (ctypes.c_int, [ctypes.c_int]),
    "scgib_set2set_save_floats": (_I64, [_I64, _I32, _I32]),
    "scgib_set2set_fwd": (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _P, _P, _P, _P, _P, _P, _P]),
    "scgib_set2set_bwd": (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _P, _P, _P, _P, _P, _I64, _P,
                                         _P, _P, _P, _P, _P]),
    "scgib_set2set_wgrad": (ctypes.c_int, [_P, _P, _I64, _I32, _I32, _P, _P, _P, _P, _P]),
    "scgib_head_fwd": (ctypes.c_int, [_P, _I64, _I32, _P, _P, _P, _P, _I32, _I32, _P, _P, _P,
                                      _P]),
    "scgib_head_bwd": (ctypes.c_int, [_P, _P, _P, _P, _I64, _I32, _P, _P, _I32, _I32, _P, _P,
                                      _P, _P, _P, _P]),
    "scgib_bce_fwd": (ctypes.c_int, [_P, _P, _I64, _P, _P]),
    "scgib_bce_bwd": (ctypes.c_int, [_P, _P, _I64, _P, _P, _P]),
    "scgib_pool_copy": (ctypes.c_int, [_P, _I32, _P, _P, _I64, _P]),
    "scgib_pool_copy2": (ctypes.c_int, [_P, _I32, _P, _P, _I64, _P, _P, _I64, _P]),
    "scgib_stream_signal": (ctypes.c_int, [_P, _P]),
    "scgib_stamp": (ctypes.c_int, [_P, _I32, _P]),
    "scgib_stream_wait": (ctypes.c_int, [_P, _P, _P, _P]),
    "scgib_graph_split": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P]),
    "scgib_graph_split_launch": (ctypes.c_int, [_P, _P]),
    "scgib_graph_split_destroy": (ctypes.c_int, [_P]),
    "scgib_graph_split_plan": (ctypes.c_int, [_I32, _I32, _P, _P, _I32, _P, _P, _P, _P, _P, _P,
                                              _P]),
    "scgib_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "scgib_gin_aggregate": (ctypes.c_int, [_P, _P, _P, _I64, _I32, _F, _P, _P, _P]),
    "scgib_segment_sum": (ctypes.c_int, [_P, _P, _I64, _I32, _P, _P, _P]),
    "scgib_segment_broadcast": (ctypes.c_int, [_P, _P, _I64, _I32, _P, _I64, _P, _P]),
    "scgib_egonet_workspace_bytes": (_I64, [_I64]),
    "scgib_egonet_count": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _I32, _I32, _P, _P, _P, _P, _P,
                                          _P]),
    "scgib_egonet_k1_max_degree": (_I64, []),
    "scgib_egonet_k1_max_graph_nodes": (_I64, []),
    "scgib_egonet_k1_build": (ctypes.c_int, [_P, _P, _I64, _P, _P, _P, _P, _P, _P, _I64, _P, _P,
                                             _P]),
    "scgib_egonet_k1_build_deg": (ctypes.c_int, [_P, _P, _I64, _I32, _P, _P, _P, _P, _P, _P, _I64,
                                                 _P, _P, _P]),
    "scgib_egonet_k1_scan_words": (_I64, [_I64]),
    "scgib_egonet_count_pool": (ctypes.c_int, [_P, _I32, _P, _I64, _I64, _I64, _I64, _I64, _I64,
                                               _I32, _I32, _P, _P, _P, _P, _P]),
    "scgib_egonet_fill_pool": (ctypes.c_int, [_P, _I32, _P, _I64, _I64, _I64, _I64, _I64, _I64,
                                              _I32, _I32, _P, _P, _P, _P, _P, _P, _I64, _P, _P]),
    "scgib_egonet_k1_build_onepass_pool": (ctypes.c_int, [_P, _I32, _P, _I64, _I64, _I64, _I64,
                                                           _I32, _P, _P, _P, _P, _P, _P, _I64,
                                                           _I64, _P, _P, _P]),
    "scgib_egonet_k1_build_onepass": (ctypes.c_int, [_P, _P, _I64, _I32, _P, _P, _P, _P, _P, _P,
                                                     _I64, _I64, _P, _P, _P, _P]),
    "scgib_egonet_fill": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _I32, _I32, _P, _P, _P, _P, _P,
                                         _P, _I64, _P, _P, _P]),
    "scgib_interaction_fwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I64, _I64, _P, _P, _P, _P,
                                             _F, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                             _P, _P, _I32, _P]),
    "scgib_noise_uniform": (ctypes.c_int, [_P, _P, _I64, _P, _P, _P]),
    "scgib_bn_running_update": (ctypes.c_int, [_P, _P, _I64, _F, _P, _P, _P, _P]),
    "scgib_interaction_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _P,
                                             _P, _P, _P, _F, _I32, _P, _P, _P, _P, _P, _P, _P,
                                             _P, _P, _P, _P, _I32, _P, _P]),
    "scgib_recon_logm_fwd": (ctypes.c_int, [_P, _P, _I64, _P, _P, _P, _I32, _P, _P, _P]),
    "scgib_recon_logm_bwd": (ctypes.c_int, [_P, _P, _I64, _P, _P, _I32, _P, _P, _P]),
    "scgib_contrastive_workspace_floats": (_I64, [_I64]),
    "scgib_contrastive_counters": (_I64, [_I64]),
    "scgib_contrastive_fwd": (ctypes.c_int, [_P, _P, _I64, _P, _P, _P, _P]),
    "scgib_contrastive_bwd": (ctypes.c_int, [_P, _P, _I64, _P, _P, _P, _P, _P, _P]),
    "scgib_mlp2_slab_floats": (_I64, [_I64, _I32]),
    "scgib_mlp2_recon_slab_floats": (_I64, [_I64, _I32]),
    "scgib_mlp2_fwd": (ctypes.c_int, [_P, _I32, _I64, _P, _P, _P, _P, _P, _P, _P, _P]),
    "scgib_mlp2_bwd": (ctypes.c_int, [_P, _P, _P, _I32, _P, _P, _I64, _P, _P, _P, _P, _P]),
    "scgib_mlp2_recon_ws_floats": (_I64, [_I64]),
    "scgib_mlp2_recon_fwd": (ctypes.c_int, [_P, _I32, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _I64,
                                            _P, _P, _P, _P, _P, _P]),
    "scgib_mlp2_recon_bwd": (ctypes.c_int, [_P, _P, _P, _P, _I32, _P, _P, _I64, _P, _P, _P, _P,
                                            _P, _P, _P, _P, _P, _P]),
    "scgib_mlp2_recon_contrastive_fwd": (ctypes.c_int, [_P, _I32, _I64, _P, _P, _P, _P, _P, _P,
                                                        _P, _P, _I64, _P, _P, _P, _P, _P, _P,
                                                        _I64, _P, _P, _P, _P, _P, _P]),
    "scgib_mlp2_recon_contrastive_bwd": (ctypes.c_int, [_P, _P, _P, _P, _I32, _P, _P, _I64, _P,
                                                        _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                                        _I64, _P, _P, _P, _P, _P, _P]),
    "scgib_linear_slab_floats": (_I64, [_I64]),
    "scgib_linear_fwd": (ctypes.c_int, [_P, _I64, _P, _P, _P, _P, _P]),
    "scgib_linear_bwd": (ctypes.c_int, [_P, _P, _P, _I64, _P, _P, _P, _P, _P, _P]),
    "scgib_gin_tiles": (_I64, [_I64]),
    "scgib_gin_layer0_slab_width": (_I64, []),
    "scgib_gin_layer0_fwd": (ctypes.c_int, [_P, _I32, _P, _P, _P, _P, _I64, _F, _P, _P, _P, _P,
                                            _P, _P, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P,
                                            _P, _P, _I32, _P]),
    "scgib_gin_layer0_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _I64,
                                            _P, _I32, _P, _P, _P]),
    "scgib_gin_hidden": (ctypes.c_int, [_P, _I32, _P, _P, _I64, _P, _P]),
    "scgib_gin_bn_gpart_offset": (_I64, [_I64]),
    "scgib_gin_defer_max_nodes": (_I64, []),
    "scgib_gin_bn_ws_floats": (_I64, [_I64]),
    "scgib_gin_counters": (_I64, [_I64]),
    "scgib_gin_layer_fwd_bn": (ctypes.c_int, [_P, _I32, _P, _P, _P, _I64, _F, _P, _P, _P, _P, _P,
                                              _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P,
                                              _P, _I32, _P]),
    "scgib_gin_bwd_stats_bn": (ctypes.c_int, [_P, _P, _P, _F, _P, _P, _I64, _I32, _P, _P, _P, _P,
                                              _P, _P, _P, _I32, _P]),
    "scgib_gin_bwd_stats_bn_fold": (ctypes.c_int, [_P, _P, _P, _F, _P, _P, _I64, _I32, _P, _P,
                                                   _P, _P, _P, _P, _P, _I32, _P, _P]),
    "scgib_gin_bwd_slabs": (_I64, [_I64]),
    "scgib_gin_layer_bwd_slabs": (_I64, [_I64, _I32]),
    "scgib_slab_reduce": (ctypes.c_int, [_P, _I32, _I64, _P, _P]),
    "scgib_gin_slab_floats": (_I64, [_I64, _I32]),
    "scgib_gin_layer_fwd": (ctypes.c_int, [_P, _I32, _P, _P, _P, _I64, _F, _P, _P, _P, _P, _P, _P,
                                           _P, _P, _P, _P]),
    "scgib_bn_finalize": (ctypes.c_int, [_P, _I64, _P, _P, _F, _F, _I32, _P, _P, _P, _P, _P, _P]),
    "scgib_bn_relu_apply": (ctypes.c_int, [_P, _P, _I64, _P, _P, _P, _P]),
    "scgib_gin_bwd_stats_seg_bn": (ctypes.c_int, [_P, _P, _P, _P, _P, _I64, _I32, _P, _P, _P,
                                                  _P, _P, _P, _P, _I32, _P]),
    "scgib_bn_relu_segment_sum": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _P, _P, _P, _P, _P, _P,
                                                 _P]),
    "scgib_gin_bwd_stats": (ctypes.c_int, [_P, _P, _P, _F, _P, _P, _I64, _P, _P, _P, _P]),
    "scgib_bn_bwd_finalize": (ctypes.c_int, [_P, _I64, _I32, _P, _P, _P, _P, _P]),
    "scgib_gin_layer_bwd": (ctypes.c_int, [_P, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _I64, _P,
                                           _P, _P, _I32, _P, _P, _P]),
    "scgib_gin_layer_bwd_z_slabs": (_I64, [_I64]),
    "scgib_gin_layer_bwd_z_width": (_I64, []),
    "scgib_gin_layer_bwd_z": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I64, _P, _P, _I32, _P, _P,
                                             _P, _P, _P]),
    "scgib_gin_bwd_stats_z_slabs": (_I64, [_I64]),
    "scgib_gin_bwd_stats_z": (ctypes.c_int, [_P, _P, _P, _F, _P, _P, _P, _I64, _I32, _P, _P, _P,
                                             _P, _P, _P, _P, _I32, _P, _I32, _P, _I32, _P]),
    "scgib_recon_partials_floats": (_I64, [_I64]),
    "scgib_recon_fwd": (ctypes.c_int, [_P, _P, _P, _I64, _I64, _P, _P, _P, _P, _P]),
    "scgib_recon_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I64, _P, _P, _P, _P]),
    "scgib_slab_reduce_max_jobs": (_I64, []),
    "scgib_slab_reduce_multi": (ctypes.c_int, [_P, _I32, _P]),
    "scgib_slab_reduce_multi_ex": (ctypes.c_int, [_P, _I32, _I32, _P]),
    "scgib_grad_pack_max_tensors": (_I64, []),
    "scgib_grad_pack": (ctypes.c_int, [_P, _I32, _P, _P]),
    "scgib_grad_unpack": (ctypes.c_int, [_P, _I32, _P, _F, _P]),
    "scgib_adam_max_tensors": (_I64, []),
    "scgib_adam_step": (ctypes.c_int, [_P, _I32, _D, _D, _D, _D, _D, _P, _P]),
    "scgib_adam_reduce_max_jobs": (_I64, []),
    "scgib_adam_step_reduce": (ctypes.c_int, [_P, _I32, _P, _I32, _D, _D, _D, _D, _D, _P, _P]),
}


class BnPending(ctypes.Structure):
    """scgib_bn_pending (include/scgib.h)."""
    _fields_ = [("gpart", ctypes.c_void_p), ("gamma", ctypes.c_void_p),
                ("beta", ctypes.c_void_p), ("running_mean", ctypes.c_void_p),
                ("running_var", ctypes.c_void_p), ("num_batches_tracked", ctypes.c_void_p),
                ("stat", ctypes.c_void_p), ("eps", ctypes.c_float), ("momentum", ctypes.c_float)]


class BnBwdPending(ctypes.Structure):
    """scgib_bn_bwd_pending (include/scgib.h)."""
    _fields_ = [("gpart", ctypes.c_void_p), ("dgamma", ctypes.c_void_p),
                ("dbeta", ctypes.c_void_p), ("training", ctypes.c_int32)]


class AdamTensor(ctypes.Structure):
    """scgib_adam_tensor (include/scgib.h)."""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p),
                ("exp_avg", ctypes.c_void_p), ("exp_avg_sq", ctypes.c_void_p),
                ("step", ctypes.c_void_p), ("numel", ctypes.c_int64)]

class SlabJob(ctypes.Structure):
    """scgib_slab_job (include/scgib.h)."""
    _fields_ = [("slab", ctypes.c_void_p), ("out", ctypes.c_void_p), ("width", ctypes.c_int64),
                ("n_slabs", ctypes.c_int32), ("stride", ctypes.c_int32)]


class GradSlice(ctypes.Structure):
    """scgib_grad_slice (include/scgib.h)."""
    _fields_ = [("data", ctypes.c_void_p), ("numel", ctypes.c_int64), ("offset", ctypes.c_int64)]


class RunningUpdate(ctypes.Structure):
    """scgib_running_update (include/scgib.h)."""
    _fields_ = [("stats", ctypes.c_void_p), ("graph_ptr", ctypes.c_void_p),
                ("n_graphs", ctypes.c_int64), ("momentum", ctypes.c_float),
                ("running_mean", ctypes.c_void_p), ("running_var", ctypes.c_void_p),
                ("num_batches_tracked", ctypes.c_void_p)]


ABI_VERSION = 22
STATS_STRIDE = 260
PGRAD_STRIDE = 324
HIDDEN = 64

_lib = None


class ScgibError(RuntimeError):
    pass


def load():
    """Load libscgib.so once; raises ScgibError if it is absent or broken."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ScgibError(f"{LIB_PATH} not found: the HIP extension is not built "
                         "(run __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.scgib_abi_version() != ABI_VERSION:
        raise ScgibError("libscgib.so ABI version mismatch")
    _lib = lib
    return lib


def call(name, *args):
    """Invoke an int-returning C-ABI function and raise on a non-zero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.scgib_strerror(rc).decode()
        raise ScgibError(f"{name} failed: {msg} (code {rc})")
    return rc


def query(name, *args):
    """Invoke a value-returning C-ABI function (sizes)."""
    return getattr(load(), name)(*args)
