"""Context parallelism: ring attention over the cp group, on the gfx950 attention kernels.

Same algorithm and API as the reference picotron/context_parallel/context_parallel.py:
  apply_context_parallel (:10-12), ring_attention (:14-15), RingAttentionFunc (:17-110),
  update_out_and_lse (:157-187), update_rope_for_context_parallel (:189-195).
Differences (MI355X-native, same numbers):
  * each block's forward is pico_attn_fwd (bf16 MFMA, fp32 LSE) instead of an eager O(S^2)
    matmul/softmax; the LSE merge is the pico_attn_merge kernel (same sigmoid/logsigmoid form);
  * each block's backward is pico_attn_bwd fed the GLOBAL O and LSE, accumulating dq directly in
    fp32 (PICO_ATTN_DQ_F32_ACCUM) instead of converting per block;
  * the interface keeps the reference's layout — q/k/v and the output are [B, H, S, D] (ref :14-15, caller
    ref picotron/model.py:147-150) — but internally the blocks run on [B, S, H, D] views of the same
    storage (a transpose view, no copy), the kernels' native layout;
  * the ring transport waits on its requests only (no device-wide synchronize per step).
"""
import os

import torch
import torch.distributed as dist

from .. import _lib, ops
from .. import process_group_manager as pgm
from .cp_communications import ContextCommunicate


def apply_context_parallel(model):
    os.environ["CONTEXT_PARALLEL"] = "1" if pgm.process_group_manager.cp_world_size > 1 else "0"
    return model


def ring_attention(q, k, v, sm_scale, is_causal):
    """q [B, Hq, S_local, D], k/v [B, Hkv, S_local, D] -> out [B, Hq, S_local, D] (ref :14-15: the
    reference's caller transposes its [B, S, H, D] projections to this layout and transposes the output
    back, ref picotron/model.py:139-150). Hkv may divide Hq (native GQA; the reference passes k/v already
    repeat_interleave'd to Hq heads, which works as well)."""
    if q.dim() != 4 or k.dim() != 4 or v.dim() != 4:
        raise ValueError("ring_attention: q, k, v must be [batch, heads, seqlen, head_dim]")
    out = RingAttentionFunc.apply(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), sm_scale, is_causal)
    return out.transpose(1, 2)


def update_out_and_lse(out, lse, block_out, block_lse):
    """Merge one block's (bf16 out [B,S,H,D], fp32 lse [B,H,S]) into the running fp32 (out, lse).
    Returns the new (out, lse); the first call allocates them (ref :157-187)."""
    B, S, H, D = block_out.shape
    first = out is None
    if first:
        out = torch.empty((B, S, H, D), dtype=torch.float32, device=block_out.device)
        lse = torch.empty((B, H, S), dtype=torch.float32, device=block_out.device)
    if block_out.stride(-1) != 1:
        block_out = block_out.contiguous()
    lib = _lib.load()
    _lib.check(lib.pico_attn_merge(_lib.ptr(out), _lib.ptr(lse), _lib.ptr(block_out), _lib.ptr(block_lse), B, S, H, D,
                                   _lib.i64x3(block_out.stride()[:3]), 1 if first else 0,
                                   _lib.stream_of(block_out)), "pico_attn_merge")
    return out, lse


class RingAttentionFunc(torch.autograd.Function):
    """Ring attention on [B, S_local, H, D] tensors (views allowed); `ring_attention` is the reference-layout
    entry point."""

    @staticmethod
    def forward(ctx, q, k, v, sm_scale, is_causal):
        comm = ContextCommunicate("comm")
        k_og, v_og = k, v
        out, lse = None, None
        for step in range(comm.world_size):
            if step + 1 != comm.world_size:
                next_k = comm.send_recv(k)
                next_v = comm.send_recv(v)
                comm.commit()
            if not is_causal or step <= comm.rank:
                block_out, block_lse = ops.attention_block_fwd(q, k, v, sm_scale, is_causal and step == 0)
                out, lse = update_out_and_lse(out, lse, block_out, block_lse)
            if step + 1 != comm.world_size:
                comm.wait()
                k, v = next_k, next_v
        out = out.to(q.dtype)
        ctx.save_for_backward(q, k_og, v_og, out, lse)
        ctx.sm_scale = sm_scale
        ctx.is_causal = is_causal
        return out

    @staticmethod
    def backward(ctx, dout, *args):
        q, k, v, out, lse = ctx.saved_tensors
        sm_scale, is_causal = ctx.sm_scale, ctx.is_causal
        kv_comm = ContextCommunicate("kv_comm")
        d_kv_comm = ContextCommunicate("d_kv_comm")
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        dk = dv = None
        next_dk = next_dv = None
        dout = dout.contiguous()
        for step in range(kv_comm.world_size):
            if step + 1 != kv_comm.world_size:
                next_k = kv_comm.send_recv(k)
                next_v = kv_comm.send_recv(v)
                kv_comm.commit()
            if step <= kv_comm.rank or not is_causal:
                _, bdk, bdv = ops.attention_block_bwd(dout, q, k, v, out, lse, sm_scale, is_causal and step == 0,
                                                      dq_accum=dq)
                if dk is None:
                    dk, dv = bdk.float(), bdv.float()
                else:
                    d_kv_comm.wait()
                    dk = next_dk + bdk
                    dv = next_dv + bdv
            elif step != 0:
                d_kv_comm.wait()
                dk, dv = next_dk, next_dv
            if step + 1 != kv_comm.world_size:
                kv_comm.wait()
                k, v = next_k, next_v
            next_dk = d_kv_comm.send_recv(dk)
            next_dv = d_kv_comm.send_recv(dv)
            d_kv_comm.commit()
        d_kv_comm.wait()
        return dq.to(q.dtype), next_dk.to(q.dtype), next_dv.to(q.dtype), None, None


def update_rope_for_context_parallel(cos, sin):
    """Slice the RoPE tables to this cp rank's contiguous sequence chunk (ref :189-195)."""
    seq_len, _ = cos.size()
    cp_rank, cp_world_size = pgm.cp_rank_and_size()
    assert seq_len % cp_world_size == 0, \
        f"Input sequence length ({seq_len}) must be divisible by cp_world_size ({cp_world_size})"
    size = seq_len // cp_world_size
    return cos[cp_rank * size:(cp_rank + 1) * size], sin[cp_rank * size:(cp_rank + 1) * size]
