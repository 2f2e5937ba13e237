"""ctypes binding of the gfx950 C-ABI library (include/picotron_hip.h).

The library is built in-tree by `python -m picotron_amd.build` (or `__graft_entry__.build()`).
There is deliberately no fallback: if the library is missing, or a tensor is not on a HIP device,
every op raises.
"""
import ctypes
import os

import torch

LIB_PATH = os.environ.get("PICO_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                           "libpicotron_hip.so")

# kernel ids (enum in include/picotron_hip.h)
K_RMSNORM_FWD, K_RMSNORM_BWD, K_RMSNORM_DW, K_ROPE = 1, 2, 3, 4
K_SWIGLU_FWD, K_SWIGLU_BWD, K_ATTN_FWD, K_ATTN_BWD_PRE = 5, 6, 7, 8
K_ATTN_BWD, K_ATTN_BWD_DQ, K_GRAD_ACCUM, K_CAST, K_SCALE, K_ATTN_MERGE = 9, 10, 11, 12, 13, 14
K_EMBEDDING_BWD, K_CE_FWD, K_CE_BWD, K_TRANSPOSE, K_ATTN_BWD_DKV, K_SORT_IDS, K_ADAMW = 15, 16, 17, 18, 19, 20, 21
K_ATTN_BWD_KV, K_ATTN_BWD_Q = 22, 23
KERNEL_NAMES = {
    K_RMSNORM_FWD: "rmsnorm_fwd", K_RMSNORM_BWD: "rmsnorm_bwd", K_RMSNORM_DW: "rmsnorm_dw", K_ROPE: "rope",
    K_SWIGLU_FWD: "swiglu_fwd", K_SWIGLU_BWD: "swiglu_bwd", K_ATTN_FWD: "attn_fwd",
    K_ATTN_BWD_PRE: "retired_8", K_ATTN_BWD: "retired_9", K_ATTN_BWD_DQ: "retired_10",
    K_GRAD_ACCUM: "grad_accum", K_CAST: "cast_f32_bf16", K_SCALE: "scale_f32", K_ATTN_MERGE: "attn_merge",
    K_EMBEDDING_BWD: "embedding_bwd", K_CE_FWD: "cross_entropy_fwd", K_CE_BWD: "cross_entropy_bwd",
    K_TRANSPOSE: "transpose_bf16", K_ATTN_BWD_DKV: "attn_bwd_dkv", K_SORT_IDS: "sort_ids", K_ADAMW: "adamw",
    K_ATTN_BWD_KV: "attn_bwd_kv", K_ATTN_BWD_Q: "attn_bwd_q",
}

# kernel-selection knobs (pico_select; PICO_SEL_* in include/picotron_hip.h)
SEL_AUTO = -1
SEL_ATTN_KVP, SEL_KVP_WAVES, SEL_ATTN_GROUPS, SEL_ATTN_FWD = 0, 1, 2, 3

ATTN_DQ_F32_ACCUM = 1
ATTN_ROPE_BWD = 2
ATTN_ROPE_Q_FWD = 4

c_i64 = ctypes.c_int64
c_vp = ctypes.c_void_p


class AttnArgs(ctypes.Structure):
    """Mirror of `pico_attn_args`."""
    _fields_ = [
        ("q", c_vp), ("k", c_vp), ("v", c_vp), ("o", c_vp), ("lse", c_vp), ("dout", c_vp),
        ("dq", c_vp), ("dk", c_vp), ("dv", c_vp), ("workspace", c_vp),
        ("batch", c_i64), ("seqlen_q", c_i64), ("seqlen_k", c_i64), ("heads_q", c_i64),
        ("heads_kv", c_i64), ("head_dim", c_i64),
        ("q_strides", c_i64 * 3), ("k_strides", c_i64 * 3), ("v_strides", c_i64 * 3), ("o_strides", c_i64 * 3),
        ("do_strides", c_i64 * 3), ("dq_strides", c_i64 * 3), ("dk_strides", c_i64 * 3), ("dv_strides", c_i64 * 3),
        ("softmax_scale", ctypes.c_float), ("causal", ctypes.c_int), ("flags", ctypes.c_int),
        ("rope_cos", c_vp), ("rope_sin", c_vp), ("rope_stride", c_i64), ("o_t", c_vp), ("o_t_ld", c_i64),
    ]


# name -> (restype, argtypes)
_SIGNATURES = {
    "pico_abi_version": (ctypes.c_int, []),
    "pico_last_error": (ctypes.c_char_p, []),
    "pico_prof_enable": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "pico_prof_collect": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_i64)]),
    "pico_select": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "pico_rmsnorm_fwd": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, ctypes.c_float, c_vp]),
    "pico_rmsnorm_fwd_t": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64,
                                          ctypes.c_float, c_vp]),
    "pico_rmsnorm_bwd_workspace_bytes": (c_i64, [c_i64, c_i64]),
    "pico_rmsnorm_bwd": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp]),
    "pico_rmsnorm_bwd_acc": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_float,
                                            c_vp, c_i64, c_i64, c_vp]),
    "pico_rmsnorm_bwd_chain": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.c_int, ctypes.c_float,
                                              c_vp, c_i64, c_i64, ctypes.c_int, c_vp, c_i64, c_i64, c_vp, ctypes.c_int,
                                              ctypes.c_float, c_vp]),
    "pico_rmsnorm_bwd_partial_rows": (c_i64, [c_i64, c_i64]),
    "pico_rmsnorm_dw_reduce": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, ctypes.c_int, ctypes.c_float, c_vp]),
    "pico_rope": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64,
                                 ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), c_i64, ctypes.c_int, c_vp]),
    "pico_swiglu_fwd": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "pico_swiglu_fwd_t": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "pico_swiglu_bwd": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "pico_attn_args_size": (c_i64, []),
    "pico_attn_fwd": (ctypes.c_int, [ctypes.POINTER(AttnArgs), c_vp]),
    "pico_attn_bwd_workspace_bytes": (c_i64, [ctypes.POINTER(AttnArgs)]),
    "pico_attn_bwd": (ctypes.c_int, [ctypes.POINTER(AttnArgs), c_vp]),
    "pico_attn_merge": (ctypes.c_int, [c_vp, ctypes.POINTER(c_i64), c_vp, ctypes.POINTER(c_i64), c_vp,
                                       ctypes.POINTER(c_i64), ctypes.c_int, c_vp, ctypes.POINTER(c_i64), c_i64, c_i64,
                                       c_i64, c_i64, ctypes.c_int, c_vp]),
    "pico_grad_accum": (ctypes.c_int, [c_vp, c_vp, c_i64, ctypes.c_float, c_vp]),
    "pico_scale_f32": (ctypes.c_int, [c_vp, c_i64, ctypes.c_float, c_vp]),
    "pico_cast_f32_bf16": (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp]),
    "pico_embedding_bwd": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, ctypes.c_int, ctypes.c_float, c_vp]),
    "pico_sort_ids": (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "pico_adamw_chunk_elems": (c_i64, []),
    "pico_adamw_bf16": (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double, c_i64, c_vp]),
    "pico_cross_entropy_fwd": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "pico_cross_entropy_fwd_grad": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "pico_ce_count": (ctypes.c_int, [c_vp, c_i64, c_i64, ctypes.c_float, c_vp, c_vp]),
    "pico_ce_mean": (ctypes.c_int, [c_vp, c_i64, c_vp, ctypes.c_float, c_vp, ctypes.c_int, c_vp, c_vp]),
    "pico_ce_scale_grad": (ctypes.c_int, [c_vp, c_i64, c_vp, ctypes.c_int, c_vp, c_vp]),
    "pico_cross_entropy_bwd": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp]),
    "pico_transpose_bf16": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_i64, c_i64, c_vp]),
}

EXPORTED_SYMBOLS = tuple(_SIGNATURES)

_lib = None


def load():
    """Load (once) and return the ctypes library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"picotron_amd: HIP library not found at {LIB_PATH}; "
                               "build it with `python -m picotron_amd.build`")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        # the selection knobs take their environment values now, at load (the first pico_select initialises the
        # table; the second puts the value back)
        lib.pico_select(SEL_ATTN_KVP, lib.pico_select(SEL_ATTN_KVP, SEL_AUTO))
        _lib = lib
    return _lib


def check(rc, op):
    if rc != 0:
        msg = load().pico_last_error().decode(errors="replace")
        raise RuntimeError(f"{op} failed (status {rc}): {msg}")


def stream_of(t: torch.Tensor):
    """The caller's current HIP stream for the tensor's device, as a void*."""
    if t.device.type != "cuda":
        raise RuntimeError(f"picotron_amd kernels need tensors on a HIP device, got {t.device}")
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def i64x3(vals):
    return (c_i64 * 3)(*[int(v) for v in vals])


def select(knob: int, value: int) -> int:
    """Set a kernel-selection knob (SEL_*; value SEL_AUTO = the library's shape rule); returns the previous value.
    The environment variables of the same names are read once, when the library loads."""
    old = load().pico_select(knob, value)
    if old == -2:
        raise ValueError(f"pico_select: unknown knob {knob}")
    return old


def prof_enable(kernel_id: int, capacity: int = 4096):
    check(load().pico_prof_enable(kernel_id, capacity), "pico_prof_enable")


def prof_collect(kernel_id: int):
    """Returns (total_ms, launches) of the enabled kernel since enable/last collect."""
    tot = ctypes.c_double(0.0)
    n = c_i64(0)
    check(load().pico_prof_collect(kernel_id, ctypes.byref(tot), ctypes.byref(n)), "pico_prof_collect")
    return tot.value, n.value
