"""Hot-path ops on the gfx950 kernels, with the signatures of the third-party calls they replace.

The reference imports three flash-attn entry points (ref picotron/model.py:7-9):
    from flash_attn.flash_attn_interface import flash_attn_func
    from flash_attn.layers.rotary import apply_rotary_emb
    from flash_attn.ops.triton.layer_norm import layer_norm_fn
This module exports functions of the same names and argument meanings, so the reference's own
model.py runs on MI355X by swapping those three imports. Unsupported options
(dropout, bias, interleaved rotary, windows, ...) raise NotImplementedError instead of silently
doing something else, and every op raises if its inputs are not bf16 tensors on a HIP device.

Extra entry points used by picotron_amd's own modules:
    swiglu(gate, up)                          - F.silu(gate) * up      (ref picotron/model.py:185)
    attention_block_fwd / attention_block_bwd - ring-attention block fwd/bwd with fp32 LSE
                                                (ref picotron/context_parallel/context_parallel.py:112-155)
"""
import contextlib
import ctypes
import math
import os
import weakref

import torch
from torch.optim.optimizer import register_optimizer_step_post_hook as _register_step_post_hook

from . import _lib

_BF16 = torch.bfloat16


def _need(t, name, dtype=_BF16):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name}: picotron_amd kernels need HIP tensors, got device {t.device}")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")


# --------------------------------------------------------------------------------------------
# RMSNorm  (flash_attn.ops.triton.layer_norm.layer_norm_fn with is_rms_norm=True)
# --------------------------------------------------------------------------------------------
class _RMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, eps, prenorm, want_t=False, pair=None):
        """pair: (xt_for, dy_for) paired-wgrad hints (wgrad_pair): the (weight, N, K) of the projection that reads
        y (its x^T goes into that projection's pair buffer) and of the projection whose output is x (dx goes into
        its dy pair buffer), or None."""
        _need(x, "x")
        _need(weight, "weight")
        # a chained dw left pending while no backward pass runs means the pass that created it raised before its
        # end-of-pass flush ran: drop it. A forward inside a running backward (activation recompute,
        # a forward from a hook) leaves it alone: that pass's next norm backward or its flush reduces it.
        if _NORM_PENDING and not _backward_running():
            _NORM_PENDING.pop(x.device, None)
        shape = x.shape
        cols = shape[-1]
        x2 = x.reshape(-1, cols).contiguous()
        rows = x2.shape[0]
        lib = _lib.load()
        y = torch.empty_like(x2)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        res2 = None
        res_out = None
        if residual is not None:
            _need(residual, "residual")
            res2 = residual.reshape(-1, cols).contiguous()
            res_out = torch.empty_like(x2)
        w = weight.contiguous()
        yt = None
        if want_t and os.getenv("PICO_XT_WGRAD", "1") != "0" and cols in (1024, 2048) and rows % 32 == 0 and \
                all(t is None or t.data_ptr() % 16 == 0 for t in (x2, res2, w)):
            # y^T as a by-product for the next projection's TT wgrad GEMM (no separate transpose pass), into the
            # projection's x^T pair buffer when its weight gradients are paired
            yt = _pair_xt(pair[0] if pair else None, cols, rows, x) if pair else None
            if yt is None:
                yt = torch.empty((cols, rows), dtype=x.dtype, device=x.device)
            _lib.check(lib.pico_rmsnorm_fwd_t(_lib.ptr(x2), _lib.ptr(res2), _lib.ptr(w), _lib.ptr(y), _lib.ptr(res_out),
                                              _lib.ptr(rstd), _lib.ptr(yt), yt.stride(0), rows, cols, float(eps),
                                              _lib.stream_of(x)), "pico_rmsnorm_fwd_t")
        else:
            _lib.check(lib.pico_rmsnorm_fwd(_lib.ptr(x2), _lib.ptr(res2), _lib.ptr(w), _lib.ptr(y), _lib.ptr(res_out),
                                            _lib.ptr(rstd), rows, cols, float(eps), _lib.stream_of(x)),
                       "pico_rmsnorm_fwd")
        x_eff = res_out if res_out is not None else x2
        ctx.save_for_backward(x_eff, w, rstd)
        ctx.weight_param = weight if weight.requires_grad else None
        ctx.shape = shape
        ctx.has_residual = residual is not None
        ctx.prenorm = prenorm
        ctx.pair_dy = pair[1] if pair else None
        y = y.view(shape)
        if yt is not None:
            y._pico_t = yt
        if prenorm:
            return y, (res_out if res_out is not None else x2).view(shape)
        return y

    @staticmethod
    def backward(ctx, dy, *rest):
        x_eff, w, rstd = ctx.saved_tensors
        cols = ctx.shape[-1]
        rows = x_eff.shape[0]
        dy2 = dy.reshape(-1, cols).contiguous()
        dres = None
        if ctx.prenorm and rest and rest[0] is not None:
            dres = rest[0].reshape(-1, cols).contiguous()
        lib = _lib.load()
        dx = _pair_dy(ctx.pair_dy, rows, cols, x_eff)  # the producing projection's dy pair buffer (wgrad_pair)
        if dx is None:
            dx = torch.empty_like(x_eff)
        mode, target, scale, ready = _norm_grad_target(ctx.weight_param, w)
        dw = target if mode == 0 else None
        ws = torch.empty(lib.pico_rmsnorm_bwd_workspace_bytes(rows, cols), dtype=torch.uint8, device=dy.device)
        # chained dw (one launch per norm): an in-place accumulation (mode 1 / 2) leaves its partial rows for the
        # next norm backward of this pass to reduce; this launch reduces the previous one's
        dev = dy.device
        prev = _NORM_PENDING.pop(dev, None)
        # (not with a readiness callback: the DP bucket's post-backward callback, queued before ours, would wait
        # for a bucket whose last norm weight is still pending)
        defer = mode != 0 and ready is None and _norm_chain_enabled()
        _lib.check(lib.pico_rmsnorm_bwd_chain(
            _lib.ptr(dy2), _lib.ptr(dres), _lib.ptr(x_eff), _lib.ptr(w), _lib.ptr(rstd), _lib.ptr(dx), _lib.ptr(target),
            mode, float(scale), _lib.ptr(ws), rows, cols, 0 if defer else 1,
            _lib.ptr(prev[0]) if prev else None, prev[1] if prev else 0, prev[2] if prev else 0,
            _lib.ptr(prev[3]) if prev else None, prev[4] if prev else 0, float(prev[5]) if prev else 1.0,
            _lib.stream_of(dy)), "pico_rmsnorm_bwd")
        if prev is not None and prev[6] is not None:
            prev[6]()  # the previous norm's weight gradient is complete now (DP bucket readiness)
        if defer:
            _NORM_PENDING[dev] = (ws, lib.pico_rmsnorm_bwd_partial_rows(rows, cols), cols, target, mode, scale, ready)
            torch.autograd.Variable._execution_engine.queue_callback(lambda: _flush_norm_dw(dev))
        elif ready is not None:
            ready()
        dx = dx.view(ctx.shape)
        return dx, (dx if ctx.has_residual else None), dw, None, None, None, None


# device -> a norm backward's dw partial rows waiting for the next norm backward of the same pass to reduce them
# (workspace, partial rows, cols, target, mode, scale, ready callback); _flush_norm_dw reduces what is left
# when the backward pass ends
_NORM_PENDING = {}


def _backward_running():
    """True on a thread that is executing an autograd backward pass (its graph task)."""
    return torch._C._current_graph_task_id() != -1


def _norm_chain_enabled():
    return os.getenv("PICO_NORM_DW_CHAIN", "1") != "0"


def _flush_norm_dw(dev):
    prev = _NORM_PENDING.pop(dev, None)
    if prev is None:
        return
    ws, nb, cols, target, mode, scale, ready = prev
    _lib.check(_lib.load().pico_rmsnorm_dw_reduce(_lib.ptr(ws), nb, cols, _lib.ptr(target), mode, float(scale),
                                                  _lib.stream_of(target)), "pico_rmsnorm_dw_reduce")
    if ready is not None:
        ready()


def _norm_grad_target(p, w):
    """Where the norm-weight gradient goes (the micro-batch accumulation folded into the dw reduction,
    as wgrad_accumulate does for the projections): (dw_mode, buffer, scale, ready-callback).
    mode 2: DataParallelBucket's fp32 main_grad += dw (x 1/W on the syncing micro-batch), then the
    bucket is told the parameter is ready; mode 1: bf16 .grad += dw in place (no DP wrapper, no hooks);
    mode 0: a fresh dw handed to autograd (first micro-batch, hooks, fusion disabled)."""
    if p is not None and wgrad_fusion_enabled() and p.is_contiguous():
        mg = getattr(p, "main_grad", None)
        if mg is not None and getattr(p, "_pico_wgrad_ready", None) is not None:
            if mg.dtype == torch.float32 and mg.is_contiguous() and mg.shape == p.shape:
                sync, world = p._pico_wgrad_sync()
                if not sync and _norm_chain_enabled():
                    # a non-syncing micro-batch: nothing waits for this bucket, so the dw reduction may be chained
                    # into the next norm backward (its readiness call only records the parameter as produced by a
                    # fused path, which must happen now, before its AccumulateGrad hook runs)
                    p._pico_wgrad_ready()
                    return 2, mg, 1.0, None
                return 2, mg, (1.0 / world if sync else 1.0), p._pico_wgrad_ready
        elif mg is None and not _has_hooks(p):
            g = p.grad
            if g is not None and g.dtype == p.dtype and g.is_contiguous() and g.shape == p.shape:
                return 1, g, 1.0, None
    return 0, torch.empty_like(w), 1.0, None


def _pair_xt(hint, K, T, like):
    """The [K, T] x^T pair-buffer slot (row stride 2T) of the projection `hint` = (weight, N, K') for the current
    micro-batch, or None (pairing off, or a shape that does not match)."""
    if hint is None:
        return None
    from . import wgrad_pair as WP
    w, N, Kh = hint
    if Kh != K or T % 8 != 0:
        return None
    return WP.xt_out(w, N, K, T, like.dtype, like.device)


def _pair_dy(hint, T, N, like):
    """The [T, N] dy pair-buffer slot of the projection `hint` = (weight, N', K) for the current micro-batch, or None."""
    if hint is None:
        return None
    from . import wgrad_pair as WP
    w, Nh, K = hint
    if Nh != N:
        return None
    # only into buffers the projection's forward created (its x^T went to the pair buffer): a path whose x^T was
    # never paired (PICO_SWIGLU_T=0, T % 64 != 0, an attention without O^T) gets no pair buffers from here
    return WP.dy_out_existing(w, N, K, T, like.dtype, like.device)


def rms_norm(x, weight, eps=1e-5, residual=None, prenorm=False):
    return _RMSNormFn.apply(x, residual, weight, eps, prenorm)


def layer_norm_fn(x, weight, bias, residual=None, x1=None, weight1=None, bias1=None, eps=1e-6, dropout_p=0.0,
                  rowscale=None, prenorm=False, residual_in_fp32=False, is_rms_norm=False,
                  return_dropout_mask=False, _emit_transposed=False, _pair=None):
    """flash-attn 2.5 `layer_norm_fn` restricted to what picotron calls: RMS norm, no bias/dropout
    (ref picotron/model.py:53-64). Returns y, or (y, residual_out) when prenorm=True."""
    if not is_rms_norm:
        raise NotImplementedError("picotron_amd.layer_norm_fn: only is_rms_norm=True is implemented")
    if bias is not None or x1 is not None or weight1 is not None or bias1 is not None or rowscale is not None:
        raise NotImplementedError("picotron_amd.layer_norm_fn: bias/x1/weight1/bias1/rowscale unsupported")
    if dropout_p != 0.0 or return_dropout_mask:
        raise NotImplementedError("picotron_amd.layer_norm_fn: dropout unsupported")
    if residual_in_fp32:
        raise NotImplementedError("picotron_amd.layer_norm_fn: residual_in_fp32 unsupported")
    return _RMSNormFn.apply(x, residual, weight, eps, prenorm, bool(_emit_transposed), _pair)


# --------------------------------------------------------------------------------------------
# Rotary embedding (flash_attn.layers.rotary.apply_rotary_emb, interleaved=False)
# --------------------------------------------------------------------------------------------
def _rope_launch(x, out, cos, sin, conjugate):
    B, S, H, D = x.shape
    lib = _lib.load()
    _lib.check(lib.pico_rope(_lib.ptr(x), _lib.ptr(out), _lib.ptr(cos), _lib.ptr(sin), B, S, H, D,
                             _lib.i64x3(x.stride()[:3]), _lib.i64x3(out.stride()[:3]), cos.stride(0),
                             1 if conjugate else 0, _lib.stream_of(x)), "pico_rope")


class _RotaryFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin):
        out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
        _rope_launch(x, out, cos, sin, False)
        ctx.save_for_backward(cos, sin)
        return out

    @staticmethod
    def backward(ctx, dout):
        cos, sin = ctx.saved_tensors
        if dout.stride(-1) != 1:
            dout = dout.contiguous()
        dx = torch.empty(dout.shape, dtype=dout.dtype, device=dout.device)
        _rope_launch(dout, dx, cos, sin, True)
        return dx, None, None


def apply_rotary_emb(x, cos, sin, interleaved=False, inplace=False, seqlen_offsets=0, cu_seqlens=None,
                     max_seqlen=None):
    """flash-attn `apply_rotary_emb`: x [B, S, H, D], cos/sin [S, D/2] (row stride free) -> [B, S, H, D]
    (ref picotron/model.py:135-136)."""
    if interleaved:
        raise NotImplementedError("picotron_amd.apply_rotary_emb: interleaved=True unsupported")
    if cu_seqlens is not None or max_seqlen is not None or (not isinstance(seqlen_offsets, int)) or seqlen_offsets:
        raise NotImplementedError("picotron_amd.apply_rotary_emb: varlen / seqlen_offsets unsupported")
    _need(x, "x")
    _need(cos, "cos")
    _need(sin, "sin")
    if x.dim() != 4:
        raise ValueError("apply_rotary_emb: x must be [batch, seqlen, heads, head_dim]")
    B, S, H, D = x.shape
    if cos.shape[0] < S or cos.shape[1] * 2 != D or sin.shape != cos.shape:
        raise ValueError(f"apply_rotary_emb: cos/sin must be [>= {S}, {D // 2}], got {tuple(cos.shape)}")
    if cos.stride(1) != 1 or sin.stride(1) != 1 or cos.stride(0) != sin.stride(0):
        raise ValueError("apply_rotary_emb: cos/sin rows must be unit-stride with equal row strides")
    if x.stride(-1) != 1:
        x = x.contiguous()
    out = _RotaryFn.apply(x, cos, sin)
    if inplace:
        with torch.no_grad():
            x.copy_(out)
        return x
    return out


# --------------------------------------------------------------------------------------------
# SwiGLU epilogue
# --------------------------------------------------------------------------------------------
def _swiglu_fwd(g, u, out, rows, cols, in_stride, out_stride):
    _lib.check(_lib.load().pico_swiglu_fwd(_lib.ptr(g), _lib.ptr(u), _lib.ptr(out), rows, cols, in_stride, out_stride,
                                           _lib.stream_of(g)), "pico_swiglu_fwd")


def _swiglu_bwd(dh, g, u, dg, du, rows, cols, in_stride, out_stride):
    _lib.check(_lib.load().pico_swiglu_bwd(_lib.ptr(dh), _lib.ptr(g), _lib.ptr(u), _lib.ptr(dg), _lib.ptr(du), rows,
                                           cols, in_stride, out_stride, _lib.stream_of(dh)), "pico_swiglu_bwd")


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gate, up):
        _need(gate, "gate")
        _need(up, "up")
        if gate.shape != up.shape:
            raise ValueError("swiglu: gate and up must have the same shape")
        g = gate.contiguous()
        u = up.contiguous()
        out = torch.empty_like(g)
        n = g.numel()
        _swiglu_fwd(g, u, out, 1, n, n, n)
        ctx.save_for_backward(g, u)
        return out

    @staticmethod
    def backward(ctx, dout):
        g, u = ctx.saved_tensors
        d = dout.contiguous()
        dg = torch.empty_like(g)
        du = torch.empty_like(u)
        n = g.numel()
        _swiglu_bwd(d, g, u, dg, du, 1, n, n, n)
        return dg, du


def swiglu(gate, up):
    """silu(gate) * up with one fused kernel each way (ref picotron/model.py:185)."""
    return _SwiGLUFn.apply(gate, up)


# --------------------------------------------------------------------------------------------
# Weight-gradient accumulation fusion (beta = 1 wgrad GEMMs)
#
# The reference accumulates micro-batch gradients outside the GEMM: autograd's AccumulateGrad does
# `p.grad += dW` in bf16 (DP = 1), and DataParallelBucket's hook does `main_grad += grad` in fp32
# (ref picotron/data_parallel/data_parallel.py:131) — one extra sweep over every parameter per
# micro-batch. Here the wgrad GEMM accumulates into the gradient's storage itself (hipBLASLt
# epilogue, beta = 1): same sums, each rounded once instead of twice, no extra sweep.
#   * DP bucket present (param.main_grad + param._pico_wgrad_ready, installed by DataParallelBucket):
#     main_grad = beta * main_grad + alpha * dW in fp32 (out_dtype), alpha = beta = 1/W on the syncing
#     micro-batch (the bucket's `grad_data /= W`, ref picotron/data_parallel/bucket.py:30, folded
#     in), then the bucket is told the param is ready. One param per GEMM (bucket views of
#     different params are not adjacent).
#   * no DP wrapper, no grad hooks: the rows of one GEMM output are the .grad of its params (views of
#     one buffer created on the first micro-batch); later micro-batches add into it with beta = 1.
#   * anything else (hooks, foreign .grad tensors, non-bf16): plain dW handed to autograd.
# --------------------------------------------------------------------------------------------
def _plain_grads(params, dW):
    out, r0 = [], 0
    for p in params:
        n = p.shape[0]
        out.append(dW[r0:r0 + n].view(p.shape))
        r0 += n
    return tuple(out)


def _has_hooks(p):
    hooks = getattr(p, "_post_accumulate_grad_hooks", None)
    return bool(hooks) or bool(getattr(p, "_backward_hooks", None))


def wgrad_fusion_enabled():
    """PICO_WGRAD_FUSION=0 restores the reference's two-step accumulation (for bitwise tests)."""
    return os.getenv("PICO_WGRAD_FUSION", "1") != "0"


def wgrad_accumulate(params, dy2, x2):
    """dW = dy2^T x2 for row-stacked `params` ([sum rows, K]); returns the grads for autograd
    (None where the GEMM already accumulated into the parameter's gradient storage)."""
    if not wgrad_fusion_enabled():
        return _plain_grads(params, torch.mm(dy2.t(), x2))
    if len(params) == 1 and getattr(params[0], "_pico_wgrad_ready", None) is not None \
            and getattr(params[0], "main_grad", None) is not None:
        p = params[0]
        mg = p.main_grad
        if mg.dtype == torch.float32 and mg.is_contiguous() and tuple(mg.shape) == tuple(p.shape):
            sync, world = p._pico_wgrad_sync()
            sc = 1.0 / world if sync else 1.0
            torch.addmm(mg, dy2.t(), x2, beta=sc, alpha=sc, out_dtype=torch.float32, out=mg)
            p._pico_wgrad_ready()
            return (None,)
    if len(params) > 1 and all(getattr(p, "_pico_wgrad_ready", None) is not None and
                               getattr(p, "main_grad", None) is not None and p.main_grad.dtype == torch.float32 and
                               p.main_grad.is_contiguous() and tuple(p.main_grad.shape) == tuple(p.shape) and
                               p.dtype == dy2.dtype for p in params):
        # Row-stacked parameters (q|k|v, gate|up) under DataParallelBucket: their main_grads sit in different
        # buckets (not one fp32 block), so one GEMM cannot accumulate into them. The reference's sequence — the
        # bf16 dW, then the bucket hook's main_grad += dW (x 1/W when syncing) — runs here, with the same kernels
        # and the same values, instead of through autograd: an AccumulateGrad node is created on the stream of
        # the forward that first uses the parameter, so in the two-stream pipelined graph (forward i + 1 beside
        # backward i) the node of micro-batch i served micro-batch i + 1 too, and torch synchronised the two
        # streams on every such gradient ("AccumulateGrad node's stream does not match ...").
        # (one fp32-output GEMM per parameter on its column slice of dy measured slower: the fp32 read-modify-write
        # then sits in the GEMM's epilogue instead of a pass the other micro-batch's work overlaps)
        from .data_parallel.bucket import get_kernels
        buf = torch.mm(dy2.t(), x2)
        r0 = 0
        for p in params:
            n = p.shape[0]
            sync, world = p._pico_wgrad_sync()
            get_kernels().accumulate(p.main_grad, buf[r0:r0 + n], world if sync else 1)
            p._pico_wgrad_ready()
            r0 += n
        return (None,) * len(params)
    if all(p.dtype == dy2.dtype and getattr(p, "main_grad", None) is None and not _has_hooks(p) for p in params):
        grads = [p.grad for p in params]
        if all(g is None for g in grads):
            buf = torch.mm(dy2.t(), x2)
            r0 = 0
            for p in params:
                n = p.shape[0]
                p.grad = buf[r0:r0 + n].view(p.shape)
                r0 += n
            return (None,) * len(params)
        if all(g is not None for g in grads):
            base = grads[0]
            nrows = sum(p.shape[0] for p in params)
            K = params[0].shape[1]
            ok = base.is_contiguous() and base.dtype == dy2.dtype
            r0 = 0
            sp = base.untyped_storage().data_ptr()
            for p, g in zip(params, grads):
                ok = ok and g.is_contiguous() and g.untyped_storage().data_ptr() == sp and \
                    g.data_ptr() == base.data_ptr() + r0 * K * base.element_size()
                r0 += p.shape[0]
            if ok:
                buf = torch.as_strided(base, (nrows, K), (K, 1))
                torch.addmm(buf, dy2.t(), x2, out=buf)
                return (None,) * len(params)
            if all(g.dtype == dy2.dtype and g.shape == p.shape for p, g in zip(params, grads)):
                # separately allocated gradients (a caller's own zeros_like per parameter): AccumulateGrad's in-place
                # `grad += dW` done here (same values), not through autograd — see the DP branch above for why
                buf = torch.mm(dy2.t(), x2)
                r0 = 0
                for p, g in zip(params, grads):
                    g.add_(buf[r0:r0 + p.shape[0]].view(p.shape))
                    r0 += p.shape[0]
                return (None,) * len(params)
    return _plain_grads(params, torch.mm(dy2.t(), x2))


# --------------------------------------------------------------------------------------------
# Transposed weight copies for the dgrad GEMMs
#
# dx = dy W runs on hipBLASLt ~7-20 % slower in that (NN) form than the same product in the forward's
# form F.linear(dy, W^T) against a contiguous W^T (measured on MI355X at M = 4096: gate_up 243 -> 213 us,
# down 117 -> 97, qkv 104 -> 97, lm_head 634 -> 588; scripts/gemm_layout_probe.py). W^T is kept per
# weight (bf16, +1 copy of the weights in HBM) and re-transposed lazily, at its next use, whenever the
# weights may have changed. Safe by default — every way a drop-in caller writes weights
# is seen:
#   * an optimizer step (a global torch.optim step post-hook bumps a generation; the fused AdamW does not
#     bump the parameters' version counters);
#   * an in-place write through the parameter itself (`with no_grad(): p.copy_(x)`, `load_state_dict`, which
#     copies into the parameters): its version counter;
#   * a parameter re-pointed at other storage (`p.data = t`, `module.to(other dtype / device)`): entries are
#     keyed by the weight's storage and data pointer.
# Not seen — and the one case that needs invalidate_weight_transposes(): an in-place write through a `.data`
# alias (`p.data.copy_(x)`, `p.data.mul_(2)`; the alias has its own version counter) and raw writes to
# p.data_ptr() by foreign kernels. Reading `.data` (logging, norms, EMA, deepcopy) costs nothing: no torch class
# is patched. MicroBatchGraph calls refresh_weight_transposes() before each replay (a replayed graph runs no host
# code). Entries hold their parameters only through weak references: a rebuilt model does not keep the old one's
# weights alive.
# --------------------------------------------------------------------------------------------
_WT_GEN = [0]
_WT_CACHE = {}  # (storage id, W.data_ptr(), shape) -> [wt, key, [weakref(p) for p in params]]
_WT_HOOK = []
_WT_STATS = {"transposes": 0}  # W^T (re)computations since import (tests: steady-state refresh count)


def _bump_wt_gen(*_):
    _WT_GEN[0] += 1


def invalidate_weight_transposes():
    """Mark every cached W^T stale (re-transposed on next use). Optimizer steps, in-place writes through the
    parameters and re-pointed parameters are detected; call this after writes through a `.data` alias
    (`p.data.copy_(x)`) or raw writes to a parameter's storage by foreign code."""
    _bump_wt_gen()


def wt_dgrad_enabled():
    """PICO_WT_DGRAD=0 computes dgrads as dy @ W (no transposed copies)."""
    return os.getenv("PICO_WT_DGRAD", "1") != "0"


def _wt_key(W):
    return (W.untyped_storage()._cdata, W.data_ptr(), tuple(W.shape))


def _wt_purge():
    for k in [k for k, e in _WT_CACHE.items() if any(r() is None for r in e[2])]:
        del _WT_CACHE[k]


def weight_t(W, params):
    """Contiguous W^T ([K, N] for W [N, K]), up to date with the parameters `params` W is made of."""
    if not _WT_HOOK:
        _WT_HOOK.append(_register_step_post_hook(_bump_wt_gen))
    key = (_WT_GEN[0],) + tuple(p._version for p in params)
    ck = _wt_key(W)
    ent = _WT_CACHE.get(ck)
    if (ent is None or ent[0].dtype != W.dtype or len(ent[2]) != len(params)
            or any(r() is not p for r, p in zip(ent[2], params))):
        _wt_purge()
        ent = [torch.empty((W.shape[1], W.shape[0]), dtype=W.dtype, device=W.device), None,
               [weakref.ref(p) for p in params]]
        _WT_CACHE[ck] = ent
    if ent[1] != key:
        with torch.no_grad():
            transpose_2d(W, out=ent[0])
        ent[1] = key
        _WT_STATS["transposes"] += 1
    return ent[0]


def transpose_2d(x, out=None):
    """Contiguous x^T ([C, R]) of a bf16 [R, C] matrix with unit column stride, on the HIP transpose
    kernel (torch's strided copy runs at ~0.5 TB/s on these shapes)."""
    R, C = x.shape
    if out is None:
        out = torch.empty((C, R), dtype=x.dtype, device=x.device)
    ok = x.dtype == _BF16 and x.stride(1) == 1 and R % 8 == 0 and C % 8 == 0 and x.stride(0) % 8 == 0 and \
        out.stride(1) == 1 and out.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0 and out.data_ptr() % 16 == 0
    if not ok:
        out.copy_(x.t())
        return out
    _need(x, "x")
    _lib.check(_lib.load().pico_transpose_bf16(_lib.ptr(x), x.stride(0), _lib.ptr(out), out.stride(0), R, C,
                                               _lib.stream_of(x)), "pico_transpose_bf16")
    return out


def _wgrad_input(x2, n_out, x=None):
    """What the backward keeps of a projection's input x2 [T, K] for its wgrad: x2 itself, or x2^T as a
    transposed view of a contiguous [K, T] copy where hipBLASLt's "TT" wgrad form saves more than the
    transpose costs (output width >= 3 K: qkv, gate|up, LM head; gemm_layout_probe.py --wgrad)."""
    if os.getenv("PICO_XT_WGRAD", "1") == "0" or not x2.is_cuda:
        return x2
    xt = getattr(x, "_pico_t", None)  # a producer wrote x^T as a by-product (attention output)
    if xt is not None and tuple(xt.shape) == (x2.shape[1], x2.shape[0]):
        return xt.t()
    if n_out >= 3 * x2.shape[1]:
        return transpose_2d(x2).t()
    return x2


def refresh_weight_transposes():
    _wt_purge()
    for ent in list(_WT_CACHE.values()):
        params = [r() for r in ent[2]]
        W = params[0].detach() if len(params) == 1 else stacked_weight(params)
        weight_t(W, params)


def dgrad(dy2, W, params):
    """dx = dy2 W for W [N, K] (the stacked weight of `params`)."""
    if wt_dgrad_enabled():
        return torch.nn.functional.linear(dy2, weight_t(W, params))
    return torch.matmul(dy2, W)


def _conc_tags():
    """PICO_WGRAD_CONC: comma list of {o (square plain projections), lin (other plain), qkv, gu, lm} or 'all' /
    'none': the wgrad GEMM of those projections runs on a side stream beside their dgrad GEMM and is joined right
    after it. Default 'gu,lm': the gate|up pair (dgrad [T, Hd] with K = 2I fills half the chip for a long K loop,
    the wgrad [2I, Hd] fills the rest) measured 866.0 -> 862.8 ms per C2 step (2 rounds x 2 boxes), the LM head's
    per-chunk pair (the same shape class, K = V) 855.5 -> 855.0 (3 rounds); the out / down / qkv pairs measured
    slower side by side (+0.5-0.9 % per step)."""
    v = os.getenv("PICO_WGRAD_CONC", "gu,lm")
    if v == "none":
        return set()
    return {"o", "lin", "qkv", "gu", "lm"} if v == "all" else set(t for t in v.split(",") if t)


_SIDE = {}
_NO_SIDE = [0]  # > 0: the dgrad / wgrad (and LM-head dx / dW) pairs run in sequence on the caller's stream


@contextlib.contextmanager
def no_side_streams():
    """Within: no side-stream fork / join in dgrad_wgrad or the chunked LM-head CE (the pipelined micro-batch
    graph, whose two micro-batches already share the chip: a fork from its forked slot stream, i.e. dependencies
    in both directions between two non-origin capture streams, crashes hipStreamEndCapture on this ROCm)."""
    _NO_SIDE[0] += 1
    try:
        yield
    finally:
        _NO_SIDE[0] -= 1


def _side_stream(dev):
    """The side stream paired with the caller's current stream on `dev` (one per (device, stream): the two
    streams of the pipelined micro-batches each fork to their own, so neither waits on the other's work)."""
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    side = _SIDE.get(key)
    if side is None:
        side = _SIDE[key] = torch.cuda.Stream(device=dev)
    return side


def _wgrad_paired(params, dy2, x2):
    """wgrad_accumulate with paired weight gradients (wgrad_pair): the first micro-batch of a pair whose operands
    sit in the pair buffers defers its GEMM (a DP readiness callback still marks the parameter as produced by a
    fused path, so the bucket hook does not add a stale .grad); the second runs one GEMM over both."""
    from . import wgrad_pair as WP
    plan = WP.plan(params[0], dy2, x2)
    if plan[0] == "skip":
        for p in params:
            ready = getattr(p, "_pico_wgrad_ready", None)
            if ready is not None and getattr(p, "main_grad", None) is not None:
                ready()
        return (None,) * len(params)
    return wgrad_accumulate(params, plan[1], plan[2])


def dgrad_wgrad(tag, dy2, W, params, x2):
    """(dx, wgrad_accumulate(...)) for one projection; concurrently on two streams when `tag` is enabled
    (joined before returning: everything after the projection's backward sees both results). Joining later
    (the next projection's backward) measured the same: the fork / join edges cost ≈ 6 + 11 µs either way."""
    if tag in _conc_tags() and dy2.is_cuda and not _NO_SIDE[0]:
        dev = dy2.device
        cur = torch.cuda.current_stream(dev)
        side = _side_stream(dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            dws = _wgrad_paired(params, dy2, x2)
        dx = dgrad(dy2, W, params)
        cur.wait_stream(side)
        return dx, dws
    return dgrad(dy2, W, params), _wgrad_paired(params, dy2, x2)


def sort_ids(flat, vocab):
    """torch.sort(flat, stable=True) of int64 token ids on pico_sort_ids (one LDS workgroup) when it fits
    (<= 8192 ids, vocab <= 2^19); the same result, bit for bit."""
    if flat.numel() > 8192 or vocab > (1 << 19) or flat.dtype != torch.int64:
        return torch.sort(flat, stable=True)
    flat = flat.contiguous()
    sids = torch.empty_like(flat)
    spos = torch.empty_like(flat)
    _lib.check(_lib.load().pico_sort_ids(_lib.ptr(flat), flat.numel(), int(vocab), _lib.ptr(sids), _lib.ptr(spos),
                                         _lib.stream_of(flat)), "pico_sort_ids")
    return sids, spos


def _embedding_bwd_into(grad, ids, dy, scale):
    flat = ids.reshape(-1)
    sids, spos = sort_ids(flat, grad.shape[0])
    dy2 = dy.reshape(-1, dy.shape[-1])
    if not dy2.is_contiguous():
        dy2 = dy2.contiguous()
    _lib.check(_lib.load().pico_embedding_bwd(_lib.ptr(sids), _lib.ptr(spos), _lib.ptr(dy2), _lib.ptr(grad),
                                              flat.numel(), dy2.shape[1], 1 if grad.dtype == torch.float32 else 0,
                                              float(scale), _lib.stream_of(dy2)), "pico_embedding_bwd")


class _EmbeddingFn(torch.autograd.Function):
    """F.embedding whose backward (pico_embedding_bwd) adds the touched rows straight into the
    gradient storage — .grad (DP = 1), or the fp32 main_grad with 1/W on the syncing micro-batch
    (DataParallelBucket) — instead of materialising a dense [V, H] gradient (ref
    picotron/model.py:223-224). Deterministic and HIP-graph safe."""

    @staticmethod
    def forward(ctx, ids, w):
        ctx.save_for_backward(ids)
        ctx.w = w
        return torch.nn.functional.embedding(ids, w)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        w = ctx.w
        if getattr(w, "_pico_wgrad_ready", None) is not None and getattr(w, "main_grad", None) is not None:
            sync, world = w._pico_wgrad_sync()
            _embedding_bwd_into(w.main_grad, ids, dy, 1.0)
            if sync and world != 1:  # the bucket's grad_data /= W covers every row, touched or not
                w.main_grad.mul_(1.0 / world)
            w._pico_wgrad_ready()
            return None, None
        if getattr(w, "main_grad", None) is None and not _has_hooks(w):
            if w.grad is None:
                w.grad = torch.zeros_like(w)
            _embedding_bwd_into(w.grad, ids, dy, 1.0)
            return None, None
        g = torch.zeros_like(w)
        _embedding_bwd_into(g, ids, dy, 1.0)
        return None, g


class _CrossEntropyFn(torch.autograd.Function):
    """F.cross_entropy(logits, target, reduction='mean') on pico_cross_entropy_fwd/_bwd: one read of
    the logits forward, one read + one write backward (ref train.py:46-49). The loss is returned in
    the logits' dtype, as ATen's is."""

    @staticmethod
    def forward(ctx, logits, target, ignore_index):
        _need(logits, "logits")
        rows, vocab = logits.shape
        if logits.stride(1) != 1:
            logits = logits.contiguous()
        t = target.reshape(-1)
        if t.dtype != torch.int64:
            t = t.long()
        t = t.contiguous()
        lse = torch.empty(rows, dtype=torch.float32, device=logits.device)
        loss_rows = torch.empty(rows, dtype=torch.float32, device=logits.device)
        _lib.check(_lib.load().pico_cross_entropy_fwd(_lib.ptr(logits), logits.stride(0), _lib.ptr(t), _lib.ptr(lse),
                                                      _lib.ptr(loss_rows), rows, vocab, int(ignore_index),
                                                      _lib.stream_of(logits)), "pico_cross_entropy_fwd")
        n_valid = (t != ignore_index).sum().to(torch.float32)  # device scalar, no host sync
        loss = loss_rows.sum() / n_valid
        ctx.save_for_backward(logits, t, lse, n_valid)
        ctx.ignore_index = int(ignore_index)
        return loss.to(logits.dtype)

    @staticmethod
    def backward(ctx, grad_out):
        logits, t, lse, n_valid = ctx.saved_tensors
        rows, vocab = logits.shape
        gscale = (grad_out.to(torch.float32) / n_valid).reshape(1).contiguous()
        dlogits = torch.empty((rows, vocab), dtype=logits.dtype, device=logits.device)
        _lib.check(_lib.load().pico_cross_entropy_bwd(_lib.ptr(logits), logits.stride(0), _lib.ptr(t), _lib.ptr(lse),
                                                      _lib.ptr(gscale), _lib.ptr(dlogits), dlogits.stride(0), rows,
                                                      vocab, ctx.ignore_index, _lib.stream_of(logits)),
                   "pico_cross_entropy_bwd")
        return dlogits, None, None


class _LMHeadCEFn(torch.autograd.Function):
    """mean F.cross_entropy(x W^T, target) in one autograd node — the LM head (ref picotron/model.py:246,
    269) and the loss (ref train.py:46-49) fused: the logits [T, V] are produced by one GEMM into a buffer
    that the CE kernel turns, in the same read, into the loss statistics AND dlogits for a unit upstream
    gradient (in place, one write). The backward only runs the two LM-head GEMMs on it, scaling their
    results by the actual upstream gradient g: dx = g (dlogits W), dW += dlogits^T (g x) — exact for any
    g (a device scalar; no host sync). Logits are never materialised twice and never re-read by a CE
    backward."""

    @staticmethod
    def forward(ctx, x, w, target, ignore_index):
        _need(x, "x")
        _need(w, "w")
        H = x.shape[-1]
        x2 = x.reshape(-1, H)
        T, V = x2.shape[0], w.shape[0]
        logits = torch.nn.functional.linear(x2, w)  # [T, V] bf16, becomes dlogits in place below
        t = target.reshape(-1)
        if t.dtype != torch.int64:
            t = t.long()
        t = t.contiguous()
        n_valid = (t != ignore_index).sum().to(torch.float32)
        gscale = (1.0 / n_valid).reshape(1)
        lse = torch.empty(T, dtype=torch.float32, device=x.device)
        loss_rows = torch.empty(T, dtype=torch.float32, device=x.device)
        _lib.check(_lib.load().pico_cross_entropy_fwd_grad(_lib.ptr(logits), logits.stride(0), _lib.ptr(t),
                                                           _lib.ptr(lse), _lib.ptr(loss_rows), _lib.ptr(gscale), T, V,
                                                           int(ignore_index), _lib.stream_of(x)),
                   "pico_cross_entropy_fwd_grad")
        loss = loss_rows.sum() / n_valid
        ctx.save_for_backward(logits, _wgrad_input(x2, V, x), w)
        ctx.xshape = x.shape
        return loss.to(x.dtype)

    @staticmethod
    def backward(ctx, grad_out):
        dlogits, xin, w = ctx.saved_tensors
        g = grad_out.to(torch.float32)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _scale_by_upstream(dgrad(dlogits, w, (w,)), grad_out).view(ctx.xshape)
        dw = None
        if ctx.needs_input_grad[1]:
            # scale the small GEMM input instead of dlogits: dW = dlogits^T (g x) (layout of x^T kept;
            # exact when g is a power of two, e.g. 1 / grad_acc)
            dw = wgrad_accumulate((w,), dlogits, xin * g)[0]
        return dx, dw, None, None


def _scale_by_upstream(dx, grad_out, nonunit=None):
    """dx (bf16, contiguous) *= the loss's upstream gradient, read on the device (pico_ce_scale_grad: same
    rounding as ATen's dx.mul_(grad_out), one streaming launch instead of a cast + a broadcasting ATen mul).
    nonunit (int32 device tensor): set to 1 by the same launch when the upstream gradient is not exactly 1."""
    if dx.dtype != torch.bfloat16 or not dx.is_contiguous() or grad_out.dtype not in (torch.bfloat16, torch.float32):
        if nonunit is not None:
            nonunit.copy_(torch.maximum(nonunit, (grad_out != 1).to(nonunit.dtype)))
        return dx.mul_(grad_out.to(torch.float32))
    g = grad_out if grad_out.is_contiguous() else grad_out.contiguous()
    _lib.check(_lib.load().pico_ce_scale_grad(_lib.ptr(dx), dx.numel(), _lib.ptr(g),
                                              1 if g.dtype == torch.float32 else 0, _lib.ptr(nonunit),
                                              _lib.stream_of(dx)), "pico_ce_scale_grad")
    return dx


# device -> int32 flag set when a chunked LM-head CE (grad_scale=...) was back-propagated with an upstream
# gradient other than 1 (its weight gradient, taken in the forward, assumed 1): read by check_lm_head_grad_scale
_CE_NONUNIT = {}


def _ce_nonunit_flag(dev):
    f = _CE_NONUNIT.get(dev)
    if f is None:
        f = _CE_NONUNIT[dev] = torch.zeros((), dtype=torch.int32, device=dev)
    return f


def check_lm_head_grad_scale(device=None):
    """Raise if any chunked lm_head_cross_entropy(grad_scale=...) since the last check received an upstream
    gradient other than exactly 1 — its dx was scaled correctly, but the weight gradient it accumulated in the
    forward was not. Reads one device int (a host sync): train_step calls it where it reads the
    loss anyway. Resets the flag."""
    for dev, f in list(_CE_NONUNIT.items()):
        if device is not None and torch.device(device) != torch.device(dev):
            continue
        if int(f.item()) != 0:
            f.zero_()
            raise RuntimeError("lm_head_cross_entropy(grad_scale=s) was back-propagated with an upstream gradient "
                               "other than 1: its weight gradient (taken in the forward for a unit upstream) is "
                               "wrong. Fold every loss scale into grad_scale and call loss.backward() on the "
                               "returned loss alone, or use the unchunked form (grad_scale=None).")


class _LMHeadCEChunkedFn(torch.autograd.Function):
    """grad_scale * mean F.cross_entropy(x W^T, target), chunked over tokens so the [T, V] logits never
    exist whole (ref picotron/model.py:246,269 + ref train.py:46-49). Per chunk of
    `chunk` rows, in the FORWARD: logits_c = x_c W^T into one reusable [chunk, V] buffer (100 MB at
    1024 x 49152 bf16, resident in the 256 MB Infinity Cache instead of a 403 MB HBM round trip), the CE
    kernel turns it in place into grad_scale * dlogits_c, then dx_c = dlogits_c W and dW += dlogits_c^T x_c
    (accumulated where wgrad_accumulate would put it: DP main_grad with 1/W folded on the syncing
    micro-batch, the bf16 .grad, or a buffer handed to autograd). The backward only scales the saved dx
    by the upstream gradient and marks the weight ready for the DP bucket.

    CONTRACT — the returned loss MUST be back-propagated with an upstream gradient of exactly 1: grad_scale is
    the gradient the loss will receive (the training loop's 1 / grad_acc folded in here instead of dividing
    the loss; loss.backward() then feeds 1). dx stays exact for any upstream gradient, but dW is accumulated
    in the forward for a unit upstream. A violation (a loss scaler, a weighted sum with another loss,
    autograd.grad with other grad_outputs) is recorded on the device by the backward's own launch and raised
    by check_lm_head_grad_scale(), which train_step runs whenever it reads the loss (PICO_CHECK_GRAD_SCALE=1
    checks inside the backward instead, with a host sync).
    loss_acc (optional fp32 0-dim device tensor): += the returned loss, inside the pico_ce_mean launch (the
    micro-batch graph's loss sum, no separate add node)."""

    @staticmethod
    def forward(ctx, x, w, target, ignore_index, grad_scale, chunk, loss_acc=None):
        _need(x, "x")
        _need(w, "w")
        H = x.shape[-1]
        x2 = x.reshape(-1, H)
        T, V = x2.shape[0], w.shape[0]
        t = target.reshape(-1)
        if t.dtype != torch.int64:
            t = t.long()
        t = t.contiguous()
        # [n_valid, grad_scale / n_valid] in one launch (pico_ce_count)
        stats = torch.empty(2, dtype=torch.float32, device=x.device)
        _lib.check(_lib.load().pico_ce_count(_lib.ptr(t), T, int(ignore_index), float(grad_scale), _lib.ptr(stats),
                                             _lib.stream_of(x)), "pico_ce_count")
        gscale = stats[1:]
        lse = torch.empty(T, dtype=torch.float32, device=x.device)
        loss_rows = torch.empty(T, dtype=torch.float32, device=x.device)
        dx = torch.empty(T, H, dtype=x.dtype, device=x.device)
        chunk = max(1, min(int(chunk), T))
        buf = None
        wt = weight_t(w, (w,)) if wt_dgrad_enabled() else None
        xin = _wgrad_input(x2, V, x)  # x2, or x2^T's transposed view ("TT" wgrad form)
        need_w = ctx.needs_input_grad[1]
        # where dW goes (wgrad_accumulate's targets), decided once for the whole call
        kind, dst, sc, ready = "autograd", None, 1.0, None
        if need_w and wgrad_fusion_enabled():
            mg = getattr(w, "main_grad", None)
            if mg is not None and getattr(w, "_pico_wgrad_ready", None) is not None:
                if mg.dtype == torch.float32 and mg.is_contiguous() and tuple(mg.shape) == tuple(w.shape):
                    sync, world = w._pico_wgrad_sync()
                    kind, dst, sc, ready = "main", mg, (1.0 / world if sync else 1.0), w._pico_wgrad_ready
            elif mg is None and not _has_hooks(w) and w.dtype == x.dtype:
                g = w.grad
                if g is None:
                    kind = "fresh"
                elif g.is_contiguous() and g.dtype == w.dtype and tuple(g.shape) == tuple(w.shape):
                    kind, dst = "grad", g
        lib = _lib.load()
        conc = "lm" in _conc_tags() and not _NO_SIDE[0]
        # grouped weight gradient (wgrad_pair's groups, one chunk per micro-batch): the logits / dlogits go into the
        # weight's dy group slot and x^T sits in its x^T slot (the final norm writes it there), and the dW GEMM runs
        # once per group, over K = r T, in the group's last micro-batch (PICO_LM_WGRAD_GROUP=0: per micro-batch)
        from . import wgrad_pair as WP
        grouped = (need_w and chunk >= T and kind in ("main", "grad") and WP.active()
                   and os.getenv("PICO_LM_WGRAD_GROUP", "1") != "0")
        if grouped:  # only when the final norm put this micro-batch's x^T into the head's group slot:
            # otherwise plan() runs a GEMM per micro-batch and a [G T, V] group buffer would be dead weight
            buf = WP.dy_out_if_paired(w, xin, V, H, T, x.dtype, x.device)
        if buf is None:
            buf = torch.empty(chunk, V, dtype=x.dtype, device=x.device)
        for c0 in range(0, T, chunk):
            c1 = min(T, c0 + chunk)
            n = c1 - c0
            lg = buf[:n]
            torch.mm(x2[c0:c1], w.t(), out=lg)
            _lib.check(lib.pico_cross_entropy_fwd_grad(_lib.ptr(lg), lg.stride(0), _lib.ptr(t[c0:c1]), _lib.ptr(lse[c0:]),
                                                       _lib.ptr(loss_rows[c0:]), _lib.ptr(gscale), n, V,
                                                       int(ignore_index), _lib.stream_of(x)),
                       "pico_cross_entropy_fwd_grad")
            # the chunk's dW GEMM on the side stream beside its dx GEMM when PICO_WGRAD_CONC has "lm" (joined
            # before the next chunk overwrites the logits buffer)
            side = None
            if conc and need_w:
                side = _side_stream(x.device)
                side.wait_stream(torch.cuda.current_stream(x.device))
            if need_w and grouped:
                plan = WP.plan(w, lg, xin)
                if plan[0] == "gemm":
                    with (torch.cuda.stream(side) if side is not None else contextlib.nullcontext()):
                        if kind == "main":  # the group's sum in one fp32 GEMM, 1/W folded in when syncing
                            torch.addmm(dst, plan[1].t(), plan[2], beta=sc, alpha=sc, out_dtype=torch.float32, out=dst)
                        else:
                            torch.addmm(dst, plan[1].t(), plan[2], out=dst)
            elif need_w:
                xc = xin[c0:c1]
                with (torch.cuda.stream(side) if side is not None else contextlib.nullcontext()):
                    if kind == "main":  # fp32 main_grad: 1/W folds into the first chunk's beta and every alpha
                        torch.addmm(dst, lg.t(), xc, beta=(sc if c0 == 0 else 1.0), alpha=sc, out_dtype=torch.float32,
                                    out=dst)
                    elif kind in ("grad", "fresh_acc", "autograd_acc"):
                        torch.addmm(dst, lg.t(), xc, out=dst)
                    elif kind == "fresh":
                        w.grad = dst = torch.mm(lg.t(), xc)
                        kind = "fresh_acc"
                    else:  # "autograd": a buffer handed back from the backward
                        dst = torch.mm(lg.t(), xc)
                        kind = "autograd_acc"
            if ctx.needs_input_grad[0]:
                if wt is not None:
                    torch.mm(lg, wt.t(), out=dx[c0:c1])
                else:
                    torch.mm(lg, w, out=dx[c0:c1])
            if side is not None:
                torch.cuda.current_stream(x.device).wait_stream(side)
        loss = torch.empty((), dtype=x.dtype, device=x.device)
        if loss_acc is not None:
            _need(loss_acc, "loss_acc", torch.float32)
        _lib.check(lib.pico_ce_mean(_lib.ptr(loss_rows), T, _lib.ptr(stats), float(grad_scale), _lib.ptr(loss),
                                    1 if x.dtype == torch.float32 else 0, _lib.ptr(loss_acc), _lib.stream_of(x)),
                   "pico_ce_mean")
        ctx.save_for_backward(dx)
        ctx.xshape = x.shape
        ctx.dw = dst if kind == "autograd_acc" else None
        ctx.ready = ready
        return loss

    @staticmethod
    def backward(ctx, grad_out):
        (dx,) = ctx.saved_tensors
        if os.getenv("PICO_CHECK_GRAD_SCALE", "0") == "1":
            assert float(grad_out) == 1.0, f"lm_head_cross_entropy(grad_scale=...): upstream gradient {float(grad_out)} != 1"
        dxo = None
        flag = _ce_nonunit_flag(dx.device)
        if ctx.needs_input_grad[0]:
            dxo = _scale_by_upstream(dx, grad_out, flag).view(ctx.xshape)
        else:
            flag.copy_(torch.maximum(flag, (grad_out != 1).to(flag.dtype)))
        if ctx.ready is not None:
            ctx.ready()
        dw = ctx.dw
        ctx.dw = None
        return dxo, dw, None, None, None, None, None


def ce_chunk_rows():
    """Rows per LM-head CE chunk in the training loop (PICO_CE_CHUNK; 0 = the unchunked fused form)."""
    return int(os.getenv("PICO_CE_CHUNK", "4096"))


def lm_head_cross_entropy(x, w, target, ignore_index=-100, grad_scale=None, chunk=None, loss_acc=None):
    """mean cross-entropy of the LM head x W^T against target, fused. grad_scale=None: the drop-in form
    (_LMHeadCEFn, logits [T, V] kept for the backward GEMMs; exact for any upstream gradient).
    grad_scale=s: returns s * mean CE, computed chunk rows at a time with dx and dW in the forward
    (_LMHeadCEChunkedFn). !! The returned loss MUST then be back-propagated with an upstream gradient of
    exactly 1 (plain loss.backward() on it alone) — the weight gradient is taken in the forward; a violation
    raises at the next check_lm_head_grad_scale() (train_step runs it). loss_acc: see _LMHeadCEChunkedFn."""
    if grad_scale is None:
        if loss_acc is not None:
            raise ValueError("lm_head_cross_entropy: loss_acc needs the chunked form (grad_scale=...)")
        return _LMHeadCEFn.apply(x, w, target, ignore_index)
    return _LMHeadCEChunkedFn.apply(x, w, target, ignore_index, float(grad_scale),
                                    ce_chunk_rows() if chunk is None else int(chunk), loss_acc)


def cross_entropy(logits, target, ignore_index=-100, reduction="mean"):
    """F.cross_entropy for [N, V] bf16 logits on a HIP device (mean reduction)."""
    if reduction != "mean":
        raise NotImplementedError("picotron_amd.cross_entropy: only reduction='mean'")
    if logits.dim() != 2:
        raise ValueError("picotron_amd.cross_entropy: logits must be [N, V]")
    return _CrossEntropyFn.apply(logits, target, ignore_index)


def embedding(ids, w):
    if not wgrad_fusion_enabled():
        return torch.nn.functional.embedding(ids, w)
    return _EmbeddingFn.apply(ids, w)


class _LinearFn(torch.autograd.Function):
    """y = x W^T (bias-free nn.Linear) whose backward folds the micro-batch gradient accumulation
    into the wgrad GEMM (wgrad_accumulate)."""

    @staticmethod
    def forward(ctx, x, w):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.save_for_backward(_wgrad_input(x2, w.shape[0], x) if ctx.needs_input_grad[1] else x2, w)
        ctx.xshape = x.shape
        return torch.nn.functional.linear(x, w)

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if ctx.needs_input_grad[0] and ctx.needs_input_grad[1]:
            dx, (dw,) = dgrad_wgrad("o" if w.shape[0] == w.shape[1] else "lin", dy2, w, (w,), x2)
            return dx.view(ctx.xshape), dw
        dx = dgrad(dy2, w, (w,)).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        dw = _wgrad_paired((w,), dy2, x2)[0] if ctx.needs_input_grad[1] else None
        return dx, dw


def linear(x, w):
    return _LinearFn.apply(x, w)


# --------------------------------------------------------------------------------------------
# Stacked weights for the fused GEMMs: [Wq; Wk; Wv] and [Wg; Wu] are one buffer whose row blocks ARE
# the parameters (p.data re-pointed in place on first use, or after a .to() moved them), so the
# fused GEMM reads the parameters themselves: no concatenated copy, nothing to refresh after the
# optimizer step, and the parameter objects, names and registration order are unchanged.
# --------------------------------------------------------------------------------------------
def stacked_weight(ws):
    K = ws[0].shape[1]
    N = sum(w.shape[0] for w in ws)
    base = ws[0]
    ok = all(w.is_contiguous() and w.dtype == base.dtype and w.device == base.device and w.shape[1] == K
             for w in ws)
    sp = base.untyped_storage().data_ptr()
    off = 0
    for w in ws:
        ok = ok and w.untyped_storage().data_ptr() == sp and \
            w.data_ptr() == base.data_ptr() + off * K * base.element_size()
        off += w.shape[0]
    if not ok:
        with torch.no_grad():
            buf = torch.cat([w.detach() for w in ws], 0)
        r0 = 0
        for w in ws:
            n = w.shape[0]
            w.data = buf[r0:r0 + n]
            r0 += n
        base = ws[0]
    return base.detach().as_strided((N, K), (K, 1))


class _GateUpSwiGLUFn(torch.autograd.Function):
    """h = silu(x Wg^T) * (x Wu^T) with ONE GEMM against [Wg; Wu] and the strided SwiGLU kernel on
    its two column halves; the backward writes dgate/dup into the halves of one [T, 2I] gradient,
    so x's gradient is one GEMM (no sum of two dgrads) and the weight gradient one GEMM."""

    @staticmethod
    def forward(ctx, x, w_gate, w_up, down_hint=None):
        """down_hint: (weight, N, K) of the down projection reading h (wgrad_pair: h^T into its x^T pair buffer)."""
        _need(x, "x")
        I = w_gate.shape[0]
        W = stacked_weight((w_gate, w_up))
        x2 = x.reshape(-1, x.shape[-1])
        gu = torch.matmul(x2, W.t())  # [T, 2I]
        T = gu.shape[0]
        h = torch.empty((T, I), dtype=x.dtype, device=x.device)
        ht = None
        if os.getenv("PICO_XT_WGRAD", "1") != "0" and os.getenv("PICO_SWIGLU_T", "1") != "0" and T % 64 == 0 \
                and I % 64 == 0 and gu.data_ptr() % 16 == 0:
            # h^T as a by-product (the down projection's wgrad reads it in the TT GEMM form)
            ht = _pair_xt(down_hint, I, T, x)
            if ht is None:
                ht = torch.empty((I, T), dtype=x.dtype, device=x.device)
            _lib.check(_lib.load().pico_swiglu_fwd_t(_lib.ptr(gu), _lib.ptr(gu[:, I:]), _lib.ptr(h), _lib.ptr(ht), T, I,
                                                     2 * I, I, ht.stride(0), _lib.stream_of(gu)), "pico_swiglu_fwd_t")
        else:
            _swiglu_fwd(gu, gu[:, I:], h, T, I, 2 * I, I)
        ctx.save_for_backward(_wgrad_input(x2, 2 * I, x), gu, W)
        ctx.params = (w_gate, w_up)
        ctx.xshape = x.shape
        out = h.view(*x.shape[:-1], I)
        if ht is not None:
            out._pico_t = ht
        return out

    @staticmethod
    def backward(ctx, dh):
        x2, gu, W = ctx.saved_tensors
        I = gu.shape[1] // 2
        d = dh.reshape(-1, I)
        if not d.is_contiguous():
            d = d.contiguous()
        from . import wgrad_pair as WP
        dgu = WP.dy_out_if_paired(ctx.params[0], x2, 2 * I, x2.shape[1], gu.shape[0], gu.dtype, gu.device)
        if dgu is None:
            dgu = torch.empty_like(gu)
        _swiglu_bwd(d, gu, gu[:, I:], dgu, dgu[:, I:], gu.shape[0], I, 2 * I, I)
        dx, (dwg, dwu) = dgrad_wgrad("gu", dgu, W, ctx.params, x2)
        return dx.view(ctx.xshape), dwg, dwu, None


def gate_up_swiglu(x, w_gate, w_up, down_hint=None):
    return _GateUpSwiGLUFn.apply(x, w_gate, w_up, down_hint)


# --------------------------------------------------------------------------------------------
# Flash attention
# --------------------------------------------------------------------------------------------
def _attn_args(q, k, v, o, lse, scale, causal):
    a = _lib.AttnArgs()
    a.q, a.k, a.v = _lib.ptr(q), _lib.ptr(k), _lib.ptr(v)
    a.o, a.lse = _lib.ptr(o), _lib.ptr(lse)
    B, Sq, Hq, D = q.shape
    a.batch, a.seqlen_q, a.heads_q, a.head_dim = B, Sq, Hq, D
    a.seqlen_k, a.heads_kv = k.shape[1], k.shape[2]
    a.q_strides = _lib.i64x3(q.stride()[:3])
    a.k_strides = _lib.i64x3(k.stride()[:3])
    a.v_strides = _lib.i64x3(v.stride()[:3])
    a.o_strides = _lib.i64x3(o.stride()[:3])
    a.softmax_scale = float(scale)
    a.causal = 1 if causal else 0
    a.flags = 0
    return a


def _check_qkv(q, k, v):
    for t, n in ((q, "q"), (k, "k"), (v, "v")):
        _need(t, n)
        if t.dim() != 4:
            raise ValueError(f"flash attention: {n} must be [batch, seqlen, heads, head_dim]")
        if t.stride(-1) != 1:
            raise ValueError(f"flash attention: {n} must have unit last-dim stride")
    if k.shape != v.shape or q.shape[0] != k.shape[0] or q.shape[3] != k.shape[3]:
        raise ValueError("flash attention: incompatible q/k/v shapes")
    if q.shape[3] not in (64, 128):
        raise NotImplementedError(f"flash attention: head_dim {q.shape[3]} unsupported (64, 128)")
    if q.shape[2] % k.shape[2] != 0:
        raise ValueError("flash attention: heads_q must be a multiple of heads_kv")


def attention_block_fwd(q, k, v, softmax_scale, causal, o_t=None, rope_q=None):
    """O [B,Sq,Hq,D] bf16 and LSE [B,Hq,Sq] fp32 (natural log) of softmax(scale*QK^T [+causal]) V.
    o_t (optional, bf16 [Hq*D, >= B*Sq] with unit column stride) also receives O transposed.
    rope_q = (cos, sin) ([>= S, D/2] bf16 tables): q is UNROTATED; the kernel applies RoPE to it in
    registers and writes the rotated queries back into q in place (PICO_ATTN_ROPE_Q_FWD)."""
    _check_qkv(q, k, v)
    if rope_q is not None and (q.stride(-1) != 1 or any(s % 8 for s in q.stride()[:3])):
        raise ValueError("attention_block_fwd: rope_q rotates q in place; q needs unit last stride and "
                         "strides that are multiples of 8")
    q, k, v = [t if t.stride(-1) == 1 and all(s % 8 == 0 for s in t.stride()[:3]) else t.contiguous()
               for t in (q, k, v)]
    B, Sq, Hq, D = q.shape
    o = torch.empty((B, Sq, Hq, D), dtype=q.dtype, device=q.device)
    lse = torch.empty((B, Hq, Sq), dtype=torch.float32, device=q.device)
    a = _attn_args(q, k, v, o, lse, softmax_scale, causal)
    if o_t is not None:
        _need(o_t, "o_t")
        if o_t.shape[0] != Hq * D or o_t.stride(1) != 1 or o_t.shape[1] < B * Sq:
            raise ValueError("attention_block_fwd: o_t must be [Hq*D, >= B*Sq] with unit column stride")
        a.o_t, a.o_t_ld = _lib.ptr(o_t), o_t.stride(0)
    if rope_q is not None:
        cos, sin = rope_q
        _check_rope_tables(cos, sin, D)
        a.flags |= _lib.ATTN_ROPE_Q_FWD
        a.rope_cos, a.rope_sin, a.rope_stride = _lib.ptr(cos), _lib.ptr(sin), cos.stride(0)
        a.dq, a.dq_strides = _lib.ptr(q), _lib.i64x3(q.stride()[:3])
    _lib.check(_lib.load().pico_attn_fwd(ctypes.byref(a), _lib.stream_of(q)), "pico_attn_fwd")
    return o, lse


def attention_block_bwd(dout, q, k, v, o, lse, softmax_scale, causal, dq_accum=None):
    """(dq, dk, dv) of attention given the (possibly global) O and LSE. If dq_accum (fp32
    [B,Sq,Hq,D]) is given, dq is ADDED into it and returned instead of a bf16 dq."""
    _check_qkv(q, k, v)
    _need(dout, "dout")
    if dout.stride(-1) != 1 or any(s % 8 for s in dout.stride()[:3]):
        dout = dout.contiguous()
    B, Sq, Hq, D = q.shape
    dk = torch.empty(k.shape, dtype=k.dtype, device=k.device)
    dv = torch.empty(v.shape, dtype=v.dtype, device=v.device)
    a = _attn_args(q, k, v, o, lse, softmax_scale, causal)
    a.dout = _lib.ptr(dout)
    a.do_strides = _lib.i64x3(dout.stride()[:3])
    if dq_accum is not None:
        _need(dq_accum, "dq_accum", torch.float32)
        dq = dq_accum
        a.flags = _lib.ATTN_DQ_F32_ACCUM
    else:
        dq = torch.empty((B, Sq, Hq, D), dtype=q.dtype, device=q.device)
    a.dq, a.dk, a.dv = _lib.ptr(dq), _lib.ptr(dk), _lib.ptr(dv)
    a.dq_strides = _lib.i64x3(dq.stride()[:3])
    a.dk_strides = _lib.i64x3(dk.stride()[:3])
    a.dv_strides = _lib.i64x3(dv.stride()[:3])
    lib = _lib.load()
    ws = torch.empty(lib.pico_attn_bwd_workspace_bytes(ctypes.byref(a)), dtype=torch.uint8, device=q.device)
    a.workspace = _lib.ptr(ws)
    _lib.check(lib.pico_attn_bwd(ctypes.byref(a), _lib.stream_of(q)), "pico_attn_bwd")
    return dq, dk, dv


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, softmax_scale, causal):
        o, lse = attention_block_fwd(q, k, v, softmax_scale, causal)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.softmax_scale = softmax_scale
        ctx.causal = causal
        return o

    @staticmethod
    def backward(ctx, dout):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = attention_block_bwd(dout, q, k, v, o, lse, ctx.softmax_scale, ctx.causal)
        return dq, dk, dv, None, None


def flash_attn_func(q, k, v, dropout_p=0.0, softmax_scale=None, causal=False, window_size=(-1, -1),
                    alibi_slopes=None, deterministic=False, return_attn_probs=False):
    """flash-attn `flash_attn_func`: q [B,Sq,Hq,D], k/v [B,Sk,Hkv,D] -> out [B,Sq,Hq,D]
    (ref picotron/model.py:32-36)."""
    if dropout_p != 0.0:
        raise NotImplementedError("picotron_amd.flash_attn_func: dropout unsupported")
    if tuple(window_size) != (-1, -1) or alibi_slopes is not None or return_attn_probs:
        raise NotImplementedError("picotron_amd.flash_attn_func: window/alibi/return_attn_probs unsupported")
    if softmax_scale is None:
        softmax_scale = 1.0 / math.sqrt(q.shape[-1])
    return _FlashAttnFn.apply(q, k, v, float(softmax_scale), bool(causal))


class _QKVRopeAttentionFn(torch.autograd.Function):
    """The attention block's hot path in one autograd node:
      qkv = x [Wq; Wk; Wv]^T (ONE GEMM) -> RoPE in place on the k columns (one launch) -> flash attention
      reading q/k/v as strided views of qkv, rotating q in registers and storing it back into qkv.
    Backward: attention writes dq/dk/dv straight into the column blocks of one dqkv buffer with RoPE^-1
    applied inside it (dQ slab sum, dK epilogue), then dx = dqkv W (one GEMM, no sum of three dgrads) and
    dW = dqkv^T x (one GEMM, rows = dWq | dWk | dWv)."""

    @staticmethod
    def forward(ctx, x, wq, wk, wv, cos, sin, nh, nkv, causal, out_hint=None):
        """out_hint: (weight, N, K) of the out-projection reading O (wgrad_pair: O^T into its x^T pair buffer)."""
        _need(x, "x")
        B, S, Hd = x.shape
        D = wq.shape[0] // nh
        W = stacked_weight((wq, wk, wv))
        N = W.shape[0]
        x2 = x.reshape(B * S, Hd)
        qkv = torch.matmul(x2, W.t())  # [T, (nh + 2 nkv) D]
        heads = qkv.view(B, S, N // D, D)
        q, k, v = heads[:, :, :nh], heads[:, :, nh:nh + nkv], heads[:, :, nh + nkv:]
        # RoPE: k in place by the rope kernel; q inside the attention forward, which writes the rotated
        # q back into qkv for the backward (PICO_FUSE_ROPE_Q=0: q|k in one rope launch, for A/B)
        fuse_q = os.getenv("PICO_FUSE_ROPE_Q", "1") != "0"
        qk = k if fuse_q else heads[:, :, : nh + nkv]  # row stride N
        _rope_launch(qk, qk, cos, sin, False)
        scale = 1.0 / math.sqrt(D)
        # O^T for the out-projection's wgrad (TT form), written by the attention epilogue for free
        o_t = None
        if os.getenv("PICO_XT_WGRAD", "1") != "0":
            o_t = _pair_xt(out_hint, nh * D, B * S, x)
            if o_t is None:
                o_t = torch.empty((nh * D, B * S), dtype=x.dtype, device=x.device)
        o, lse = attention_block_fwd(q, k, v, scale, causal, o_t=o_t, rope_q=(cos, sin) if fuse_q else None)
        ctx.save_for_backward(_wgrad_input(x2, N, x), W, qkv, o, lse, cos, sin)
        ctx.params = (wq, wk, wv)
        ctx.meta = (B, S, Hd, nh, nkv, D, causal, scale)
        out = o.view(B, S, nh * D)
        if o_t is not None:
            out._pico_t = o_t
        return out

    @staticmethod
    def backward(ctx, do):
        x2, W, qkv, o, lse, cos, sin = ctx.saved_tensors
        B, S, Hd, nh, nkv, D, causal, scale = ctx.meta
        N = W.shape[0]
        heads = qkv.view(B, S, N // D, D)
        q, k, v = heads[:, :, :nh], heads[:, :, nh:nh + nkv], heads[:, :, nh + nkv:]
        from . import wgrad_pair as WP
        # the q|k|v dy pair buffer when the forward paired this micro-batch's x^T (wgrad_pair)
        dqkv = WP.dy_out_if_paired(ctx.params[0], x2, N, Hd, B * S, qkv.dtype, qkv.device)
        if dqkv is None:
            dqkv = torch.empty_like(qkv)
        dheads = dqkv.view(B, S, N // D, D)
        # RoPE^-1 on dq | dk fused into the attention backward's dQ sum and dK epilogue
        # (PICO_FUSE_ROPE_BWD=0: separate in-place rope launch, for A/B)
        fused = os.getenv("PICO_FUSE_ROPE_BWD", "1") != "0"
        _attention_bwd_into(do.reshape(B, S, nh, D), q, k, v, o, lse, scale, causal,
                            dheads[:, :, :nh], dheads[:, :, nh:nh + nkv], dheads[:, :, nh + nkv:],
                            rope=(cos, sin) if fused else None)
        if not fused:
            dqk = dheads[:, :, : nh + nkv]
            _rope_launch(dqk, dqk, cos, sin, True)
        dx, (dwq, dwk, dwv) = dgrad_wgrad("qkv", dqkv, W, ctx.params, x2)
        return dx.view(B, S, Hd), dwq, dwk, dwv, None, None, None, None, None, None


def qkv_rope_attention(x, wq, wk, wv, cos, sin, num_heads, num_kv_heads, causal, out_hint=None):
    """Fused attention block (projections + RoPE + flash attention); see _QKVRopeAttentionFn."""
    D = wq.shape[0] // num_heads
    return _QKVRopeAttentionFn.apply(x, wq, wk, wv, cos[:, : D // 2], sin[:, : D // 2], num_heads, num_kv_heads,
                                     causal, out_hint)


def _check_rope_tables(cos, sin, D):
    _need(cos, "cos")
    _need(sin, "sin")
    if cos.stride(1) != 1 or sin.stride(1) != 1 or sin.stride(0) != cos.stride(0) or cos.shape[1] * 2 != D:
        raise ValueError("attention rope: cos/sin must be [>= S, D/2] with unit column stride")


def _attention_bwd_into(dout, q, k, v, o, lse, softmax_scale, causal, dq, dk, dv, rope=None):
    """attention backward writing into caller-provided (possibly strided) dq/dk/dv. rope = (cos, sin)
    ([>= S, D/2] bf16 tables): q and k were rotated before the forward; dq and dk come back rotated by
    -theta (the RoPE backward fused into the dQ sum and the dK epilogue, PICO_ATTN_ROPE_BWD)."""
    if dout.stride(-1) != 1 or any(s_ % 8 for s_ in dout.stride()[:3]):
        dout = dout.contiguous()
    a = _attn_args(q, k, v, o, lse, softmax_scale, causal)
    a.dout = _lib.ptr(dout)
    a.do_strides = _lib.i64x3(dout.stride()[:3])
    a.dq, a.dk, a.dv = _lib.ptr(dq), _lib.ptr(dk), _lib.ptr(dv)
    a.dq_strides = _lib.i64x3(dq.stride()[:3])
    a.dk_strides = _lib.i64x3(dk.stride()[:3])
    a.dv_strides = _lib.i64x3(dv.stride()[:3])
    if rope is not None:
        cos, sin = rope
        _check_rope_tables(cos, sin, q.shape[3])
        a.flags |= _lib.ATTN_ROPE_BWD
        a.rope_cos, a.rope_sin, a.rope_stride = _lib.ptr(cos), _lib.ptr(sin), cos.stride(0)
    lib = _lib.load()
    ws = torch.empty(lib.pico_attn_bwd_workspace_bytes(ctypes.byref(a)), dtype=torch.uint8, device=q.device)
    a.workspace = _lib.ptr(ws)
    _lib.check(lib.pico_attn_bwd(ctypes.byref(a), _lib.stream_of(q)), "pico_attn_bwd")
