"""ORACLE — TEST INFRASTRUCTURE ONLY. Never imported by the product package (picotron_amd/).

CPU restatement (torch on CPU, fp32/fp64) of the reference's hot path, used as the checker by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg. Each function cites the
reference file:line it restates (ref = rkinas/picotron @ /root/reference, not present on the GPU
box). Pinned against golden vectors produced by importing the reference itself in the build
container (tests/golden/make_golden.py -> tests/golden/*.safetensors; see tests/test_oracle.py).

The flash-attn 2.5.0 CUDA/Triton kernels the reference calls on GPU are not available anywhere
here; their fused numerics (single-rounding RMSNorm/rotary) are restated from flash-attn's
published algorithm and are "parity unpinned" beyond the eager-path goldens.
"""
import math

import torch
import torch.nn.functional as F


# ---------------------------------------------------------------------------------------------
# RoPE
# ---------------------------------------------------------------------------------------------
def get_cos_sin(seq_length, head_dim, base=500000.0, dtype=torch.bfloat16):
    """ref picotron/model.py:21-30 with DEVICE=cpu: theta in fp32 on CPU, cos/sin of
    position*theta in fp32, cast to `dtype`, repeated twice along the last dim -> [S, D]."""
    assert head_dim % 2 == 0
    theta = 1.0 / (base ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    position = torch.arange(seq_length).unsqueeze(1).float()
    ang = position.float() * theta.float()
    return torch.cos(ang).to(dtype).repeat(1, 2), torch.sin(ang).to(dtype).repeat(1, 2)


def rope_eager(x, cos, sin):
    """ref picotron/model.py:12-19 (x [B, H, S, D], tables [S, D]); arithmetic in x's dtype."""
    d = x.size(-1)
    x1, x2 = x[..., : d // 2], x[..., d // 2:]
    return x * cos + torch.cat([-x2, x1], dim=-1) * sin


def rope_fused(x, cos, sin, conjugate=False):
    """flash-attn apply_rotary_emb(interleaved=False) numerics on x [B, S, H, D] with tables
    [S, >= D/2]: fp32 math on the bf16 inputs, one rounding to x.dtype. conjugate=True rotates by
    -theta (the backward)."""
    d = x.size(-1)
    S = x.size(1)
    ct = torch.float64 if x.dtype == torch.float64 else torch.float32
    c = cos[:S, : d // 2].to(ct)[None, :, None, :]
    s = sin[:S, : d // 2].to(ct)[None, :, None, :]
    if conjugate:
        s = -s
    xf = x.to(ct)
    x1, x2 = xf[..., : d // 2], xf[..., d // 2:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(x.dtype)


# ---------------------------------------------------------------------------------------------
# RMSNorm
# ---------------------------------------------------------------------------------------------
def rmsnorm_eager(x, w, eps):
    """LlamaRMSNorm.forward, ref picotron/model.py:80-85 (normalise in fp32, round, then * w)."""
    dt = x.dtype
    h = x.to(torch.float32)
    var = h.pow(2).mean(-1, keepdim=True)
    h = h * torch.rsqrt(var + eps)
    return w * h.to(dt)


def rmsnorm_fused(x, w, eps, residual=None):
    """layer_norm_fn(is_rms_norm=True) numerics (ref picotron/model.py:53-64): optional residual
    added and rounded to x.dtype, statistic and weight product in fp32, one rounding.
    Returns (y, x_eff)."""
    xe = x if residual is None else (x.float() + residual.float()).to(x.dtype)
    h = xe.float()
    rstd = torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps)
    return (h * rstd * w.float()).to(x.dtype), xe


def rmsnorm_grads(x, w, eps, dy):
    """Exact (fp64) gradients of y = x * rsqrt(mean(x^2)+eps) * w: returns (dx, dw)."""
    xd = x.double().detach().requires_grad_(True)
    wd = w.double().detach().requires_grad_(True)
    y = xd * torch.rsqrt(xd.pow(2).mean(-1, keepdim=True) + eps) * wd
    y.backward(dy.double())
    return xd.grad, wd.grad


# ---------------------------------------------------------------------------------------------
# SwiGLU
# ---------------------------------------------------------------------------------------------
def swiglu(g, u):
    """ref picotron/model.py:185 epilogue F.silu(g) * u, computed in fp32 (fp64 for fp64 inputs)."""
    ct = torch.float64 if g.dtype == torch.float64 else torch.float32
    return F.silu(g.to(ct)) * u.to(ct)


def swiglu_grads(g, u, dh):
    """fp64 (dg, du) of h = silu(g) * u."""
    gd = g.double().detach().requires_grad_(True)
    ud = u.double().detach().requires_grad_(True)
    (F.silu(gd) * ud).backward(dh.double())
    return gd.grad, ud.grad


# ---------------------------------------------------------------------------------------------
# Attention (ring-attention block primitives; whole-sequence attention = one block)
# ---------------------------------------------------------------------------------------------
def _expand_kv(k, hq):
    """GQA: repeat_interleave kv heads to hq heads (ref picotron/model.py:141-142); k [B, H, S, D]."""
    g = hq // k.size(1)
    return k.repeat_interleave(g, dim=1) if g > 1 else k


def attention_fwd(q, k, v, sm_scale, causal):
    """ring_attention_forward, ref picotron/context_parallel/context_parallel.py:112-128.
    q [B, Hq, Sq, D], k/v [B, Hkv, Sk, D] -> (O [B, Hq, Sq, D], LSE [B, Hq, Sq]) in q's dtype/fp32."""
    k = _expand_kv(k, q.size(1))
    v = _expand_kv(v, q.size(1))
    S = torch.matmul(q, k.transpose(-2, -1)) * sm_scale
    if causal:
        sq, sk = q.size(2), k.size(2)
        mask = torch.triu(torch.ones(sq, sk, dtype=torch.bool), diagonal=1)
        S = S.masked_fill(mask, float("-inf"))
    m = S.max(dim=-1, keepdim=True)[0]
    e = torch.exp(S - m)
    ssum = e.sum(dim=-1, keepdim=True)
    lse = torch.log(ssum) + m
    return torch.matmul(e / ssum, v), lse.squeeze(-1)


def attention_bwd(dO, q, k, v, O, lse, sm_scale, causal):
    """ring_attention_backward, ref .../context_parallel.py:130-155 (recompute P from LSE; GQA:
    dk/dv summed over the query heads sharing a kv head)."""
    hkv = k.size(1)
    kx = _expand_kv(k, q.size(1))
    vx = _expand_kv(v, q.size(1))
    S = torch.matmul(q, kx.transpose(-2, -1)) * sm_scale
    if causal:
        mask = torch.triu(torch.ones(q.size(2), k.size(2), dtype=torch.bool), diagonal=1)
        S = S.masked_fill(mask, float("-inf"))
    P = torch.exp(S - lse.unsqueeze(-1))
    dV = torch.matmul(P.transpose(-2, -1), dO)
    dP = torch.matmul(dO, vx.transpose(-2, -1))
    D = torch.sum(dO * O, dim=-1, keepdim=True)
    dS = P * (dP - D)
    if causal:
        dS = dS.masked_fill(mask, 0)
    dQ = torch.matmul(dS, kx) * sm_scale
    dK = torch.matmul(dS.transpose(-2, -1), q) * sm_scale
    g = q.size(1) // hkv
    if g > 1:
        B, _, Sk, Dd = dK.shape
        dK = dK.view(B, hkv, g, Sk, Dd).sum(2)
        dV = dV.view(B, hkv, g, Sk, Dd).sum(2)
    return dQ, dK, dV


def update_out_and_lse(out, lse, block_out, block_lse, slice_=None):
    """ref .../context_parallel.py:157-187 (sigmoid/logsigmoid merge; out fp32, lse [..., 1]; slice_ merges
    into out[slice_] / lse[slice_] only, :183-184)."""
    def _update(current_out, current_lse):
        current_out = current_out - F.sigmoid(block_lse - current_lse) * (current_out - block_out)
        current_lse = current_lse - F.logsigmoid(current_lse - block_lse)
        return current_out, current_lse

    block_out = block_out.to(torch.float32)
    block_lse = block_lse.unsqueeze(dim=-1)
    if out is None:
        if slice_ is not None:
            raise RuntimeError("first update_out_and_lse should not pass slice_ args")
        return block_out, block_lse
    if slice_ is not None:
        out[slice_], lse[slice_] = _update(out[slice_], lse[slice_])
    else:
        out, lse = _update(out, lse)
    return out, lse


# ---------------------------------------------------------------------------------------------
# Data-parallel buckets
# ---------------------------------------------------------------------------------------------
def bucket_layout(numels, requires_grad, bucket_size):
    """BucketManager._initialize_buckets, ref picotron/data_parallel/bucket.py:84-116, as pure
    integer arithmetic: returns ([(start, end, bucket_idx) | None per param], bucket_sizes)."""
    locs = []
    cur, idx = 0, 0
    for n, rg in zip(numels, requires_grad):
        if not rg:
            locs.append(None)
            continue
        if cur == 0:
            locs.append((0, n, idx))
            cur = n
            continue
        if cur + n > bucket_size:
            idx += 1
            locs.append((0, n, idx))
            cur = n
        else:
            locs.append((cur, cur + n, idx))
            cur += n
    sizes = [0] * (idx + 1) if any(l is not None for l in locs) else []
    for l in locs:
        if l is not None:
            sizes[l[2]] = max(sizes[l[2]], l[1])
    return locs, sizes


def bucket_size_elems(bucket_cap_mb=25, grad_type=torch.float32):
    """ref picotron/data_parallel/data_parallel.py:81-82."""
    grad_size = 2 if grad_type == torch.bfloat16 else 4
    return bucket_cap_mb * 1024 * 1024 // grad_size


class CpuBucketKernels:
    """CPU device-op table for picotron_amd.data_parallel.bucket in gloo tests: exactly the
    reference's ATen ops (add_ then /=, ref data_parallel.py:131 / bucket.py:30; .to(dtype) :165).
    (On CPU ATen divides; on a GPU it multiplies by fp32(1/W) — equal for power-of-two W.)"""

    @staticmethod
    def accumulate(main_grad, grad, divide_by):
        main_grad.add_(grad)
        if divide_by != 1:
            main_grad /= divide_by

    @staticmethod
    def scale(buf, divide_by):
        if divide_by != 1:
            buf /= divide_by

    @staticmethod
    def cast(src, dst):
        dst.copy_(src.to(dst.dtype))

    @staticmethod
    def zero(buf):
        buf.zero_()


# ---------------------------------------------------------------------------------------------
# Model-level FLOP accounting (ref picotron/utils.py:42-48)
# ---------------------------------------------------------------------------------------------
def flops_per_token(num_params, num_layers, hidden, seq_len):
    return 6 * num_params + 12 * num_layers * hidden * seq_len


def attention_flops(batch, heads, seqlen, head_dim, causal=True, backward=False):
    """Algorithmic MFMA FLOPs of one attention call: fwd 4*B*H*S^2*D (x1/2 causal), bwd 2.5x fwd."""
    f = 4.0 * batch * heads * seqlen * seqlen * head_dim
    if causal:
        f /= 2
    return f * (2.5 if backward else 1.0)


def ln_v(vocab):
    return math.log(vocab)
