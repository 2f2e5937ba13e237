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
  * the ring transport waits on its requests only (no device-wide synchronize per step);
  * optional zig-zag load balancing (PICO_CP_ZIGZAG=1; the reference's TODO at
    ref tests/test_dataloader.py:136): the sequence is cut into 2 * cp chunks and cp rank r holds chunks
    r and 2 cp - 1 - r, so with a causal mask every rank does the same work at every ring step — the
    reference's contiguous split leaves rank r with r + 1 of cp block products (rank cp - 1 does cp,
    rank 0 one). The loader (data.py), the RoPE slice (update_rope_for_context_parallel) and the ring
    (RingAttentionFunc) switch together; zigzag_positions() is the one definition of the layout.
"""
import os

import torch
import torch.distributed as dist

from .. import _lib, ops
from .. import process_group_manager as pgm
from .cp_communications import ContextCommunicate


def apply_context_parallel(model, zigzag=None):
    """ref :10-12 (sets CONTEXT_PARALLEL). zigzag=True/False also switches the sequence layout; the decoder
    layers' RoPE tables, sliced when the model was built, are re-sliced for the layout now in force, so the
    reference's order (build the model, then apply CP, ref train.py:175-188) rotates every rank's rows by
    their global positions."""
    os.environ["CONTEXT_PARALLEL"] = "1" if pgm.process_group_manager.cp_world_size > 1 else "0"
    if zigzag is not None:
        os.environ["PICO_CP_ZIGZAG"] = "1" if zigzag else "0"
    for m in model.modules():
        refresh = getattr(m, "refresh_rope", None)
        if callable(refresh):
            refresh()
    return model


def zigzag_enabled():
    return os.getenv("PICO_CP_ZIGZAG", "0") == "1"


def zigzag_positions(seq_len, cp_rank, cp_world_size):
    """Global token positions held by `cp_rank` under the zig-zag split: chunk r, then chunk 2 cp - 1 - r
    (chunk = seq_len / (2 cp)); increasing, so a causal mask over the local sequence is the global one
    restricted to it."""
    assert seq_len % (2 * cp_world_size) == 0, \
        f"zig-zag context parallelism needs seq_len ({seq_len}) divisible by 2 * cp ({2 * cp_world_size})"
    c = seq_len // (2 * cp_world_size)
    first = torch.arange(cp_rank * c, (cp_rank + 1) * c, device="cpu")
    second = torch.arange((2 * cp_world_size - 1 - cp_rank) * c, (2 * cp_world_size - cp_rank) * c, device="cpu")
    return torch.cat([first, second])


def ring_attention(q, k, v, sm_scale, is_causal):
    """q [B, Hq, S_local, D], k/v [B, Hkv, S_local, D] -> out [B, Hq, S_local, D] (ref :14-15: the
    reference's caller transposes its [B, S, H, D] projections to this layout and transposes the output
    back, ref picotron/model.py:139-150). Hkv may divide Hq (native GQA; the reference passes k/v already
    repeat_interleave'd to Hq heads, which works as well)."""
    if q.dim() != 4 or k.dim() != 4 or v.dim() != 4:
        raise ValueError("ring_attention: q, k, v must be [batch, heads, seqlen, head_dim]")
    out = RingAttentionFunc.apply(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), sm_scale, is_causal)
    return out.transpose(1, 2)


def _merge_launch(out, out_st, lse, lse_st, block_out, bo_st, block_lse, bl_st, B, S, H, D, first):
    """pico_attn_merge on element strides: out / block_out (b, s, h) with unit d stride, lse / block_lse
    (b, h, s)."""
    ops._need(block_out, "block_out", None)
    if block_out.dtype not in (torch.bfloat16, torch.float32):
        raise TypeError(f"update_out_and_lse: block_out must be bf16 or fp32, got {block_out.dtype}")
    for t, n in ((out, "out"), (lse, "lse"), (block_lse, "block_lse")):
        ops._need(t, n, torch.float32)
    _lib.check(_lib.load().pico_attn_merge(
        _lib.ptr(out), _lib.i64x3(out_st), _lib.ptr(lse), _lib.i64x3(lse_st), _lib.ptr(block_out), _lib.i64x3(bo_st),
        1 if block_out.dtype == torch.float32 else 0, _lib.ptr(block_lse), _lib.i64x3(bl_st), B, S, H, D,
        1 if first else 0, _lib.stream_of(block_out)), "pico_attn_merge")


def _merge_bshd(out, lse, block_out, block_lse):
    """The ring's internal merge: block (out [B,S,H,D], lse [B,H,S]) into the running fp32 (out [B,S,H,D],
    lse [B,H,S]); the first call allocates them. Same arithmetic as update_out_and_lse."""
    B, S, H, D = block_out.shape
    first = out is None
    if first:
        out = torch.empty((B, S, H, D), dtype=torch.float32, device=block_out.device)
        lse = torch.empty((B, H, S), dtype=torch.float32, device=block_out.device)
    if block_out.stride(-1) != 1:
        block_out = block_out.contiguous()
    _merge_launch(out, out.stride()[:3], lse, lse.stride(), block_out, block_out.stride()[:3], block_lse,
                  block_lse.stride(), B, S, H, D, first)
    return out, lse


def update_out_and_lse(out, lse, block_out, block_lse, slice_=None):
    """ref :157-187, same signature, layout and semantics: block_out [B, H, S, D], block_lse [B, H, S]; the running
    out is fp32 [B, H, S, D] and lse fp32 [B, H, S, 1].
      * first call (out None): returns (block_out as fp32, block_lse[..., None]) as new tensors; with slice_ it
        raises, as there;
      * slice_ given: merges into out[slice_] / lse[slice_] IN PLACE (the reference's slice assignment) and returns
        (out, lse);
      * otherwise: returns NEW merged tensors and leaves the caller's out / lse untouched, as the reference's
        `_update` rebinding does (one fp32 copy each; the ring itself merges in place through _merge_bshd).
    Operands of other dtypes are cast as the reference does (block_out.to(fp32) when it is neither bf16 — read
    natively by the kernel — nor fp32; block_lse and a non-slice running out / lse to fp32). Runs on
    pico_attn_merge through element strides."""
    if block_out.dim() != 4 or block_lse.dim() != 3 or tuple(block_lse.shape) != tuple(block_out.shape[:3]):
        raise ValueError("update_out_and_lse: block_out must be [B, H, S, D] and block_lse [B, H, S]")
    if block_out.dtype not in (torch.bfloat16, torch.float32):
        block_out = block_out.to(torch.float32)
    if block_lse.dtype != torch.float32:
        block_lse = block_lse.to(torch.float32)
    if block_out.stride(-1) != 1:
        block_out = block_out.contiguous()
    B, H, S, D = block_out.shape
    if out is None:
        if slice_ is not None:
            raise RuntimeError("first update_out_and_lse should not pass slice_ args")
        out = torch.empty((B, H, S, D), dtype=torch.float32, device=block_out.device)
        lse = torch.empty((B, H, S, 1), dtype=torch.float32, device=block_out.device)
        first = True
        ov, lv = out, lse
    elif slice_ is not None:
        first = False
        if out.dtype != torch.float32 or lse.dtype != torch.float32:
            raise TypeError("update_out_and_lse: an in-place (slice_) merge needs the fp32 running out / lse")
        ov, lv = out[slice_], lse[slice_]
    else:
        first = False
        out = out.to(torch.float32, copy=True)
        lse = lse.to(torch.float32, copy=True)
        ov, lv = out, lse
    if ov.dim() != 4 or tuple(ov.shape) != (B, H, S, D) or ov.stride(-1) != 1 or \
            lv.dim() != 4 or tuple(lv.shape) != (B, H, S, 1):
        raise ValueError(f"update_out_and_lse: out{'[slice_]' if slice_ is not None else ''} must be [B, H, S, D] "
                         f"with unit last stride and lse [B, H, S, 1] matching block_out {tuple(block_out.shape)}")
    # [B, H, S, D] operands addressed as (b, s, h) rows; lse as (b, h, s)
    ost, bst = ov.stride(), block_out.stride()
    _merge_launch(ov, (ost[0], ost[2], ost[1]), lv, lv.stride()[:3], block_out, (bst[0], bst[2], bst[1]),
                  block_lse, block_lse.stride(), B, S, H, D, first)
    return out, lse


class RingAttentionFunc(torch.autograd.Function):
    """Ring attention on [B, S_local, H, D] tensors (views allowed); `ring_attention` is the reference-layout
    entry point."""

    @staticmethod
    def forward(ctx, q, k, v, sm_scale, is_causal):
        comm = ContextCommunicate("comm")
        zz = is_causal and zigzag_enabled() and comm.world_size > 1
        ctx.zigzag = zz
        if zz:
            out, lse = RingAttentionFunc._zigzag_forward(comm, q, k, v, sm_scale)
            ctx.save_for_backward(q, k, v, out, lse)
            ctx.sm_scale = sm_scale
            ctx.is_causal = is_causal
            return out
        k_og, v_og = k, v
        out, lse = None, None
        for step in range(comm.world_size):
            if step + 1 != comm.world_size:
                next_k = comm.send_recv(k)
                next_v = comm.send_recv(v)
                comm.commit()
            if not is_causal or step <= comm.rank:
                block_out, block_lse = ops.attention_block_fwd(q, k, v, sm_scale, is_causal and step == 0)
                out, lse = _merge_bshd(out, lse, block_out, block_lse)
            if step + 1 != comm.world_size:
                comm.wait()
                k, v = next_k, next_v
        out = out.to(q.dtype)
        ctx.save_for_backward(q, k_og, v_og, out, lse)
        ctx.sm_scale = sm_scale
        ctx.is_causal = is_causal
        return out

    @staticmethod
    def _zigzag_forward(comm, q, k, v, sm_scale):
        """Local rows = [chunk r | chunk 2n-1-r], each c long. Step 0 (own K/V): causal over the local rows.
        K/V from rank src < r: both query chunks see src's first chunk only (its second lies after both):
        all rows x first c keys. From src > r: only the second query chunk sees anything, and all of it:
        last c rows x all keys. Every step after the first is c x 2c, on every rank."""
        c = q.shape[1] // 2
        r, n = comm.rank, comm.world_size
        halves = [[None, None], [None, None]]  # running fp32 (out, lse) of query chunks 0 and 1

        def merge(h, bo, bl):
            halves[h][0], halves[h][1] = _merge_bshd(halves[h][0], halves[h][1], bo, bl)

        for step in range(n):
            if step + 1 != n:
                next_k = comm.send_recv(k)
                next_v = comm.send_recv(v)
                comm.commit()
            src = (r - step) % n
            if step == 0 or src < r:
                kk, vv = (k, v) if step == 0 else (k[:, :c], v[:, :c])
                bo, bl = ops.attention_block_fwd(q, kk, vv, sm_scale, step == 0)
                merge(0, bo[:, :c], bl[:, :, :c])
                merge(1, bo[:, c:], bl[:, :, c:])
            else:
                bo, bl = ops.attention_block_fwd(q[:, c:], k, v, sm_scale, False)
                merge(1, bo, bl)
            if step + 1 != n:
                comm.wait()
                k, v = next_k, next_v
        out = torch.cat([halves[0][0], halves[1][0]], 1).to(q.dtype)
        lse = torch.cat([halves[0][1], halves[1][1]], 2)
        return out, lse

    @staticmethod
    def backward(ctx, dout, *args):
        q, k, v, out, lse = ctx.saved_tensors
        sm_scale, is_causal = ctx.sm_scale, ctx.is_causal
        kv_comm = ContextCommunicate("kv_comm")
        d_kv_comm = ContextCommunicate("d_kv_comm")
        if ctx.zigzag:
            return RingAttentionFunc._zigzag_backward(kv_comm, d_kv_comm, dout, q, k, v, out, lse, sm_scale)
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

    @staticmethod
    def _zigzag_backward(kv_comm, d_kv_comm, dout, q, k, v, out, lse, sm_scale):
        """Block backwards from the GLOBAL O / LSE in the forward's zig-zag pattern; the partial dK/dV of
        the K/V block in hand travels the ring with it and returns complete to its owner."""
        c = q.shape[1] // 2
        r, n = kv_comm.rank, kv_comm.world_size
        dout = dout.contiguous()
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        lse1 = lse[:, :, c:].contiguous()
        dk = dv = next_dk = next_dv = None
        for step in range(n):
            if step + 1 != n:
                next_k = kv_comm.send_recv(k)
                next_v = kv_comm.send_recv(v)
                kv_comm.commit()
            src = (r - step) % n
            if step == 0:
                _, bdk, bdv = ops.attention_block_bwd(dout, q, k, v, out, lse, sm_scale, True, dq_accum=dq)
                dk, dv = bdk.float(), bdv.float()
            else:
                if src < r:  # all local rows x the first c keys of src
                    _, bdk, bdv = ops.attention_block_bwd(dout, q, k[:, :c], v[:, :c], out, lse, sm_scale, False,
                                                          dq_accum=dq)
                else:        # the last c local rows x all keys of src
                    _, bdk, bdv = ops.attention_block_bwd(dout[:, c:], q[:, c:], k, v, out[:, c:], lse1, sm_scale,
                                                          False, dq_accum=dq[:, c:])
                d_kv_comm.wait()
                dk, dv = next_dk, next_dv
                if src < r:
                    dk[:, :c] += bdk
                    dv[:, :c] += bdv
                else:
                    dk += bdk
                    dv += bdv
            if step + 1 != n:
                kv_comm.wait()
                k, v = next_k, next_v
            next_dk = d_kv_comm.send_recv(dk)
            next_dv = d_kv_comm.send_recv(dv)
            d_kv_comm.commit()
        d_kv_comm.wait()
        return dq.to(q.dtype), next_dk.to(q.dtype), next_dv.to(q.dtype), None, None


def update_rope_for_context_parallel(cos, sin):
    """Slice the RoPE tables to this cp rank's contiguous sequence chunk (ref :189-195), or to its two
    zig-zag chunks (PICO_CP_ZIGZAG=1)."""
    seq_len, _ = cos.size()
    cp_rank, cp_world_size = pgm.cp_rank_and_size()
    if zigzag_enabled() and cp_world_size > 1:
        idx = zigzag_positions(seq_len, cp_rank, cp_world_size).to(cos.device)
        return cos.index_select(0, idx), sin.index_select(0, idx)
    assert seq_len % cp_world_size == 0, \
        f"Input sequence length ({seq_len}) must be divisible by cp_world_size ({cp_world_size})"
    size = seq_len // cp_world_size
    return cos[cp_rank * size:(cp_rank + 1) * size], sin[cp_rank * size:(cp_rank + 1) * size]
