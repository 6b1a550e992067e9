"""ctypes binding of libmmt_hip.so (C-ABI declared in include/mmt.h).

The library is the ONLY compute path: there is no CPU or PyTorch fallback. If the shared
library is missing or cannot be loaded, `lib()` raises; if no ROCm device is present, the model
raises at forward time.

torch must be imported before the library is loaded: the library links libamdhip64.so.7 and
the dynamic loader then binds it to the HIP runtime torch already loaded (one runtime per
process, shared streams and allocations).
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime first; see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
# MMT_LIB_PATH: an experimental build of the same library (tools/build_variant.py); default in-tree
LIB_PATH = os.environ.get("MMT_LIB_PATH") or os.path.join(HERE, "libmmt_hip.so")
MAX_MOD = 8

c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_f32 = ctypes.c_float
c_vp = ctypes.c_void_p
c_cp = ctypes.c_char_p


class MmtConfig(ctypes.Structure):
    _fields_ = [
        ("num_modalities", c_i32),
        ("n_embd", c_i32),
        ("n_head", c_i32),
        ("n_layer", c_i32),
        ("block_size", c_i32),
        ("vocab_sizes", c_i32 * MAX_MOD),
        ("cross_attention", c_i32 * MAX_MOD),
        ("dropout", c_f32),
        ("seed", ctypes.c_uint64),
        ("precision", c_i32),
    ]


EPI = {
    "store_bf16": 0, "bias_tanh_bf16": 1, "bias_relu_bf16": 2, "bias_resid_f32": 3, "store_f32": 4,
    "dtanh_bf16": 5, "drelu_bf16": 6, "acc_f32": 7, "atomic_f32": 8,
}

_SIGS = {
    "mmt_create": (c_vp, [ctypes.POINTER(MmtConfig)]),
    "mmt_create_error": (c_cp, []),
    "mmt_destroy": (None, [c_vp]),
    "mmt_last_error": (c_cp, [c_vp]),
    "mmt_version": (c_cp, []),
    "mmt_param_count": (c_i64, [c_vp]),
    "mmt_param_active_count": (c_i64, [c_vp]),
    "mmt_tensor_count": (c_i32, [c_vp]),
    "mmt_tensor_info": (c_i32, [c_vp, c_i32, ctypes.c_char_p, c_i32, ctypes.POINTER(c_i64), ctypes.POINTER(c_i32),
                                ctypes.POINTER(c_i64), ctypes.POINTER(c_i32)]),
    "mmt_workspace_bytes": (c_i64, [c_vp, c_i32]),
    "mmt_loss_flag_offset": (c_i64, [c_vp, c_i32]),
    "mmt_forward": (c_i32, [c_vp, c_vp, c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_vp,
                            ctypes.POINTER(c_vp), c_vp, c_vp, c_i32]),
    "mmt_backward": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mmt_decode_step": (c_i32, [c_vp, c_vp, c_i32, c_i32, ctypes.POINTER(c_vp), c_vp, ctypes.POINTER(c_vp), c_vp]),
    "mmt_backward_stage_count": (c_i32, [c_vp]),
    "mmt_backward_stage_range": (c_i32, [c_vp, c_i32, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64)]),
    "mmt_backward_stage": (c_i32, [c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "mmt_adamw_step": (c_i32, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_f32, c_f32, c_f32, c_f32, c_f32]),
    "mmt_eval_direction": (c_i32, [c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp]),
    "mmt_set_dropout_seed": (c_i32, [c_vp, ctypes.c_uint64]),
    "mmt_probe_set": (c_i32, [c_vp, c_cp]),
    "mmt_probe_read": (c_i32, [c_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_i64)]),
    "mmt_probe_enable": (c_i32, [c_vp, c_i32]),
    "mmt_set_side_stream": (c_i32, [c_vp, c_i32]),
    "mmt_probe_count": (c_i32, [c_vp]),
    "mmt_probe_read_at": (c_i32, [c_vp, c_i32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_i64),
                                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "mmt_batch_jitter":(c_i32, [c_vp, c_vp, c_i64, c_i32, c_i32, ctypes.c_uint64, ctypes.c_uint64]),
    "mmt_batch_indices": (c_i32, [c_vp, c_i32, c_vp, c_vp, c_i32, c_i32, ctypes.c_uint64, ctypes.c_uint64, c_vp]),
    "mmt_batch_gather": (c_i32, [c_vp, c_i32, ctypes.POINTER(c_vp), c_vp, c_i32, c_i32, ctypes.POINTER(c_vp),
                                 ctypes.POINTER(c_vp)]),
    "mmt_exact_words_bytes": (c_i64, [c_i64]),
    "mmt_exact_walk_scratch_bytes": (c_i64, [c_i64, c_i64]),
    "mmt_exact_gen": (c_i32, [c_vp, c_vp, c_vp, c_i64]),
    "mmt_exact_walk": (c_i32, [c_vp, c_i32, ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), ctypes.POINTER(c_i32),
                               ctypes.POINTER(c_i32), c_vp, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "mmt_attn_set_ring": (c_i32, [ctypes.c_int]),
    "mmt_attn_set_mask_g": (c_i32, [ctypes.c_int]),
    "mmt_gemm_set_t2": (c_i32, [ctypes.c_int]),
    "mmt_emb_set_sort": (c_i32, [ctypes.c_int]),
    "mmt_set_relu_bits": (c_i32, [ctypes.c_int]),
    "mmt_set_drop_copy_fuse": (c_i32, [ctypes.c_int]),
    "mmt_set_attn_qkv2": (c_i32, [ctypes.c_int]),
    "mmt_mlp2_set_bm": (c_i32, [ctypes.c_int]),
    "mmt_qkv2_set_coal": (c_i32, [ctypes.c_int]),
    "mmt_gemm_set_variant": (c_i32, [ctypes.c_int]),
    "mmt_op_gemm": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp,
                            c_vp, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp, c_i32, c_f32]),
    "mmt_op_gemm_qkv": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_i32, c_vp, c_i32,
                                c_vp, c_i32]),
    "mmt_op_gemm_wgrad": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp, c_i32, c_f32, c_vp, c_i64]),
    "mmt_op_gemm_ln_bwd": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_f32, c_vp, c_vp, c_vp, c_vp,
                                   c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_uint32, ctypes.c_uint32, c_f32]),
    "mmt_op_mlp2": (c_i32, [c_vp, c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp, c_i32, c_vp,
                            c_vp, c_vp, ctypes.c_uint32, ctypes.c_uint32, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mmt_op_mlp2_bwd": (c_i32, [c_vp, c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp, c_i32, c_f32, c_vp, c_i32, c_vp,
                                c_i32, c_vp, c_vp]),
    "mmt_op_layernorm_fwd": (c_i32, [c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mmt_op_layernorm_bwd": (c_i32, [c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mmt_op_attention_fwd": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_i32, ctypes.POINTER(c_vp),
                                     ctypes.POINTER(c_vp), c_i32, c_i32, c_vp, c_i32, ctypes.POINTER(c_vp),
                                     ctypes.POINTER(c_vp)]),
    "mmt_op_attention_bwd": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_i32, ctypes.POINTER(c_vp),
                                     ctypes.POINTER(c_vp), c_i32, c_i32, c_vp, c_i32, ctypes.POINTER(c_vp),
                                     ctypes.POINTER(c_vp), c_vp, c_i32, ctypes.POINTER(c_vp), c_vp, c_i32,
                                     ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_i32, c_i32]),
    "mmt_op_attention_bwd_ws": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_i32, ctypes.POINTER(c_vp),
                                        ctypes.POINTER(c_vp), c_i32, c_i32, c_vp, c_i32, ctypes.POINTER(c_vp),
                                        ctypes.POINTER(c_vp), c_vp, c_i32, ctypes.POINTER(c_vp), c_vp, c_i32,
                                        ctypes.POINTER(c_vp), ctypes.POINTER(c_vp), c_i32, c_i32, c_vp, c_i32]),
    "mmt_op_qkv2_fwd": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp, c_i32]),
    "mmt_op_qkv2_bwd": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp, c_i32, c_vp, c_vp]),
    "mmt_op_colsum": (c_i32, [c_vp, c_i32, c_i32, c_vp, c_i32, c_vp, c_f32]),
    "mmt_op_cross_entropy": (c_i32, [c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp]),
    "mmt_op_embedding_fwd": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "mmt_op_embedding_bwd": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp]),
    "mmt_op_embedding_bwd_ws": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mmt_op_mx_quant": (c_i32, [c_vp, c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp, c_i32]),
    "mmt_op_gemm_f8": (c_i32, [c_vp, c_i32, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp, c_i32,
                               c_vp, c_vp, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp, c_i32]),
    "mmt_op_layernorm_fwd_f8": (c_i32, [c_vp, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_vp,
                                        c_i32]),
}

EXPORTED = sorted(_SIGS)
_lib = None


def lib():
    """Load (once) and return the ctypes handle. Raises if the library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"libmmt_hip.so not found at {LIB_PATH}: build it with "
            f"`python trade-aid-multimodal-transformer_amd/mmt_build.py` (there is no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        if os.environ.get("MMT_LIB_PATH") and not hasattr(L, name):
            continue  # an older experimental build (A/B base) lacks an entry point added since
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


class MmtError(RuntimeError):
    pass


def check(rc, ctx=None, what="mmt call"):
    if rc != 0:
        msg = lib().mmt_last_error(ctx).decode() if ctx else ""
        raise MmtError(f"{what} failed (status {rc}): {msg}")


def ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def ptr_array(ts):
    arr = (ctypes.c_void_p * max(1, len(ts)))()
    for i, t in enumerate(ts):
        arr[i] = 0 if t is None else t.data_ptr()
    return arr


def stream_ptr(device=None, stream=None):
    """HIP stream handle of `stream` (default: torch's current stream on `device`)."""
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)
