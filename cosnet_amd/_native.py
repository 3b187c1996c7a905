"""ctypes binding of libcosnet_hip.so (the C ABI declared in include/cosnet_hip.h).

The library is the only compute path: if it is missing or cannot be loaded on a GPU box,
every op raises instead of falling back to anything else.  torch must be imported before
the library is loaded so that both share torch's HIP runtime (same soname).
"""
import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime the library binds to)

_HERE = os.path.dirname(os.path.abspath(__file__))
# COSNET_HIP_LIB: development override (tools/ A/B builds); the package loads the in-tree build
LIB_PATH = os.environ.get("COSNET_HIP_LIB") or os.path.join(_HERE, "_lib", "libcosnet_hip.so")

DT_F32 = 0
DT_BF16 = 1

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_longlong
_F = ctypes.c_float
_S = ctypes.c_size_t

# name -> (restype, argtypes); stream is always the last argument (void*)
_SIGS = {
    "cn_conv_fwd": (_I, [_I, _P, _L, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _I, _P, _P, _L, _I, _I, _P]),
    "cn_conv_fwd_ws": (_I, [_I, _P, _L, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _I, _P, _P, _L, _I, _I,
                            _P, _S, _P]),
    "cn_conv_fwd_workspace_floats": (_S, [_I, _I, _I, _I]),
    "cn_conv_dgrad": (_I, [_I, _P, _L, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _I, _P, _L, _I, _I, _I, _P]),
    "cn_conv_wgrad_workspace_floats": (_S, [_I, _I, _I, _I, _I, _I, _I, _I]),
    "cn_conv_wgrad": (_I, [_I, _P, _L, _I, _I, _I, _I, _P, _L, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "cn_conv_wgrad_grouped": (_I, [_I, _I, _P, _L, _I, _I, _I, _I, _P, _L, _I, _I, _I, _I, _I, _I, _I, _I,
                                   _P, _P]),
    "cn_conv_wgrad_grouped_workspace_floats": (_S, [_I, _I, _I, _I, _I, _I, _I, _I, _I]),
    "cn_conv_wgrad_grouped_ws": (_I, [_I, _I, _P, _L, _I, _I, _I, _I, _P, _L, _I, _I, _I, _I, _I, _I, _I,
                                      _I, _P, _P, _S, _P]),
    "cn_splitk_reduce": (_I, [_P, _I, _L, _L, _P, _I, _P]),
    "cn_fp8_quant": (_I, [_I, _P, _L, _I, _I, _P, _L, _P, _I, _P]),
    "cn_fp8_quant_fmt": (_I, [_I, _I, _P, _L, _I, _I, _P, _L, _P, _I, _P]),
    "cn_conv_dgrad_fp8": (_I, [_P, _L, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _P, _L, _I, _I, _I,
                               _P, _P, _P]),
    "cn_fp8_update": (_I, [_P, _I, _F, _P]),
    "cn_fp8_quant_multi": (_I, [_P, _I, _P]),
    "cn_conv_fwd_fp8": (_I, [_P, _L, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _I, _P, _P, _L, _I, _I, _P,
                             _P, _P]),
    "cn_conv_fwd_bn_workspace_floats": (_S, [_I, _I, _I, _I]),
    "cn_conv_fwd_bn_grouped": (_I, [_I, _P, _L, _I, _I, _I, _I, _I, _P, _I, _I, _I, _P, _P, _P, _L, _I,
                                    _P, _P, _P, _P, _P, _F, _F, _P]),
    "cn_conv_fwd_fp8_bn": (_I, [_P, _L, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _I, _P, _P, _L, _I, _I,
                                _P, _P, _I, _P, _P, _P, _P, _P, _F, _F, _P]),
    "cn_conv_fwd_bn": (_I, [_I, _P, _L, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _I, _P, _P, _L, _I, _I,
                            _I, _P, _P, _P, _P, _P, _F, _F, _P]),
    "cn_conv_dgrad_bn_workspace_floats": (_S, [_I, _I, _I, _I]),
    "cn_conv_dgrad_bn": (_I, [_I, _P, _L, _I, _I, _I, _I, _P, _I, _I, _I, _I, _I, _P, _L, _I, _I, _P,
                              _L, _P, _P, _P, _P, _P, _P, _P, _P]),
    "cn_bn_bwd_apply": (_I, [_I, _P, _L, _P, _L, _I, _I, _P, _P, _P, _P, _P, _P, _P, _L, _P]),
    "cn_gemm": (_I, [_I, _I, _I, _I, _I, _I, _I, _I, _P, _L, _L, _P, _L, _L, _P, _L, _L, _I, _I, _F, _P, _I, _I, _L, _P]),
    "cn_bn_workspace_floats": (_S, [_I, _I, _I, _I]),
    "cn_bn_stats": (_I, [_I, _P, _L, _I, _I, _I, _P, _P, _P, _P, _F, _F, _P, _P]),
    "cn_bn_eval_params": (_I, [_P, _P, _I, _F, _P, _P, _P]),
    "cn_bn_apply": (_I, [_I, _P, _L, _I, _I, _I, _P, _P, _P, _P, _P, _L, _P, _L, _P, _P, _P, _P, _I, _P, _P, _L, _P]),
    "cn_bn_apply_fp8": (_I, [_I, _P, _L, _I, _I, _I, _P, _P, _P, _P, _P, _L, _P, _L, _P, _P, _P, _P, _I, _P,
                             _P, _L, _P, _L, _P, _P]),
    "cn_bn_apply_ex": (_I, [_I, _P, _L, _I, _I, _I, _P, _P, _P, _P, _P, _L, _P, _L, _P, _P, _P, _P, _I, _P,
                            _P, _L, _P, _L, _P, _P, _L, _P]),
    "cn_bn_set_tuning": (_I, [_I, _I]),
    "cn_bn_bwd": (_I, [_I, _P, _L, _P, _L, _P, _L, _I, _I, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _L, _P, _L, _P, _P]),
    "cn_coatt_workspace_floats": (_S, [_I, _I, _I]),
    "cn_coatt_softmax": (_I, [_I, _P, _I, _I, _I, _P, _P, _P, _P]),
    "cn_coatt_dscore": (_I, [_I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P]),
    "cn_coatt_fused_fwd": (_I, [_P, _L, _P, _L, _P, _L, _I, _I, _I, _P, _P, _L, _P]),
    "cn_coatt_fused_fwd_ws": (_I, [_P, _L, _P, _L, _P, _L, _I, _I, _I, _P, _P, _L, _P, _S, _P]),
    "cn_coatt_fused_workspace_bytes": (_S, [_I, _I, _I]),
    "cn_coatt_f8_workspace_bytes": (_S, [_I, _I]),
    "cn_coatt_f8_fwd": (_I, [_P, _L, _P, _L, _P, _L, _I, _I, _I, _P, _P, _L, _P, _P, _P, _S, _P]),
    "cn_coatt_f8_train_workspace_bytes": (_S, [_I, _I]),
    "cn_coatt_f8_train_fwd": (_I, [_P, _L, _P, _L, _P, _L, _I, _I, _I, _P, _P, _L, _P, _P, _P, _P, _P, _L, _P, _S, _P]),
    "cn_coatt_flash_fwd": (_I, [_P, _L, _P, _L, _P, _L, _I, _I, _I, _P, _P, _L, _P, _P, _P]),
    "cn_coatt_flash_fwd_ws": (_I, [_P, _L, _P, _L, _P, _L, _I, _I, _I, _P, _P, _L, _P, _P, _P, _S, _P]),
    "cn_coatt_flash_pv": (_I, [_P, _L, _P, _L, _P, _L, _P, _I, _I, _I, _P, _L, _I, _P]),
    "cn_coatt_flash_dvat": (_I, [_P, _L, _P, _L, _P, _L, _P, _L, _P, _L, _P, _P, _P, _P, _I, _I, _I, _P,
                                 _L, _I, _P]),
    "cn_coatt_flash_dvat_ws": (_I, [_P, _L, _P, _L, _P, _L, _P, _L, _P, _L, _P, _P, _P, _P, _I, _I, _I, _P,
                                    _L, _I, _P, _S, _P]),
    "cn_coatt_flash_bwd_workspace_bytes": (_S, [_I, _I]),
    "cn_coatt_flash_pv_ws": (_I, [_P, _L, _P, _L, _P, _L, _P, _I, _I, _I, _P, _L, _I, _P, _S, _P]),
    "cn_rowdot_seg": (_I, [_I, _P, _L, _P, _L, _I, _I, _I, _I, _P, _P]),
    "cn_nchw_to_nhwc": (_I, [_I, _P, _I, _I, _I, _I, _I, _P, _P]),
    "cn_weight_prep": (_I, [_I, _P, _I, _I, _I, _I, _P, _P, _P]),
    "cn_maxpool_fwd": (_I, [_I, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "cn_maxpool_bwd": (_I, [_I, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "cn_avgpool": (_I, [_I, _P, _L, _I, _I, _I, _F, _P, _P, _P]),
    "cn_avgpool_workspace_floats": (_S, [_I, _I, _I, _I]),
    "cn_bcast_rows": (_I, [_I, _P, _I, _I, _I, _F, _P, _L, _I, _P]),
    "cn_gate_fwd": (_I, [_I, _P, _L, _I, _I, _P, _P, _P, _L, _P, _P]),
    "cn_gate_bwd": (_I, [_I, _P, _L, _P, _L, _P, _I, _I, _P, _I, _P, _L, _P, _P, _P, _P]),
    "cn_colpart_workspace_floats": (_S, [_I, _I]),
    "cn_mean_rows": (_I, [_P, _I, _I, _P, _P]),
    "cn_sum_rows": (_I, [_P, _I, _I, _P, _P]),
    "cn_scale_dev": (_I, [_P, _L, _P, _P, _P]),
    "cn_scale": (_I, [_P, _L, _F, _P]),
    "cn_soft_iou": (_I, [_P, _P, _I, _L, _P, _P, _P, _P]),
    "cn_frame_resize": (_I, [_I, _P, _I, _L, _L, _L, _I, _I, _I, _I, _P, _P, _I, _I, _I, _I, _P]),
    "cn_gemm_force_config": (_I, [_I]),
    "cn_gemm_set_wgrad_target": (_I, [_I]),
    "cn_coatt_force_variant": (_I, [_I]),
    "cn_head_fwd": (_I, [_I, _P, _L, _P, _L, _I, _I, _I, _P, _P, _P, _L, _P, _P]),
    "cn_head_bwd": (_I, [_I, _P, _L, _P, _I, _I, _I, _P, _P, _L, _P, _P, _P, _P]),
    "cn_upsample_sigmoid": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P]),
    "cn_upsample_sigmoid_bwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P, _P]),
    "cn_count_ge": (_I, [_P, _L, _F, _P, _P]),
    "cn_loss_workspace_floats": (_S, [_L]),
    "cn_bce_l1": (_I, [_P, _P, _L, _F, _F, _P, _P, _P, _P]),
    "cn_bce_l1_devcount": (_I, [_P, _P, _L, _P, ctypes.c_double, _F, _P, _P, _P, _P]),
    "cn_sgd": (_I, [_P, _I, _P, _F, _F, _P]),
    "cn_rowdot": (_I, [_I, _P, _L, _P, _L, _I, _I, _P, _P]),
    "cn_colsum": (_I, [_I, _P, _L, _I, _I, _P, _P, _P]),
    "cn_cast2d": (_I, [_I, _I, _P, _L, _I, _I, _P, _L, _I, _P]),
    "cn_build_source_hash": (ctypes.c_char_p, []),
    "cn_build_experimental": (_I, []),
    "cn_conv_wgrad_fp8_workspace_floats": (_S, [_I, _I, _I, _I, _I, _I, _I, _I]),
    "cn_conv_wgrad_fp8": (_I, [_I, _P, _L, _I, _I, _I, _I, _P, _L, _I, _I, _I, _I, _I, _I, _I, _I,
                               _P, _P, _P, _P, _S, _P]),
}

_lib = None


class NativeError(RuntimeError):
    pass


def load():
    """Load the library (once).  Raises NativeError if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError("libcosnet_hip.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        # an A/B build of an older tree (COSNET_HIP_LIB) may lack the newest entry points; the
        # in-tree product library must export every one
        if os.environ.get("COSNET_HIP_LIB") and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


HASHED_SOURCES = ["gemm.hip", "conv.hip", "bn.hip", "ew.hip", "coatt.hip", "coatt_fused.hip",
                  "coatt_q48.hip", "coatt_flash.hip", "coatt_f8.hip", "fp8.hip", "frames.hip", "eval.hip",
                  "common.h", "gemm.h", "coatt_fused.h", "../../include/cosnet_hip.h"]   # csrc/Makefile HASHED, same order


def source_hash():
    """SHA-256 (16 hex digits) of the HIP sources in this tree, as the Makefile stamps it."""
    import hashlib
    h = hashlib.sha256()
    for f in HASHED_SOURCES:
        with open(os.path.join(_HERE, "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_info():
    """{library hash stamped at build, this tree's source hash, match, library sha256}."""
    import hashlib
    lib_hash = load().cn_build_source_hash().decode()
    with open(LIB_PATH, "rb") as fh:
        so = hashlib.sha256(fh.read()).hexdigest()[:16]
    src = source_hash()
    return {"lib_source_hash": lib_hash, "tree_source_hash": src, "built_from_tree": lib_hash == src,
            "lib_sha256": so, "lib": os.path.relpath(LIB_PATH, os.path.dirname(_HERE))}


def exported_symbols():
    return sorted(_SIGS.keys())


_ERR = {-1: "shape", -2: "alignment", -3: "unsupported", -4: "hip runtime"}


def call(name, *args):
    """Invoke one C-ABI entry point; non-zero status -> NativeError."""
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise NativeError("%s failed: %s (%d)" % (name, _ERR.get(rc, "hipError"), rc))
    return rc


def query(name, *args):
    return getattr(load(), name)(*args)


def stream():
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def dtype_code(dt):
    if dt == torch.bfloat16:
        return DT_BF16
    if dt == torch.float32:
        return DT_F32
    raise NativeError("unsupported compute dtype %s" % dt)
