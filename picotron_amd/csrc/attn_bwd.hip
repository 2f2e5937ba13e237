// C-ABI entry points of the flash-attention backward (and the argument checks it shares with the forward).
//
// Replaces flash-attn's backward of flash_attn_func (ref picotron/model.py:36) and the ring block backward
// ring_attention_backward (ref picotron/context_parallel/context_parallel.py:130-155), which recomputes P from
// the (global) O and LSE:  P = exp(scale*QK^T - LSE), dV = P^T dO, dP = dO V^T, delta = rowsum(dO * O),
// dS = P * (dP - delta), dQ = scale * dS K, dK = scale * dS^T Q.
//
// The kernels are the split form for both head dims (attn_bwd_split.hip; attn_bwd_split_d128.hip for D = 128):
// a query-major dQ kernel and a key-major dK/dV kernel, each output with one owner (no atomics, no dQ slabs).
// Round 1's fused backward (one kernel per key block, per-key-block fp32 dQ slabs summed by a second pass) was
// slower at every measured shape and is gone; its kernel ids 8-10 stay reserved in
// picotron_hip.h so the profiling ids of the others do not move.
#include "attn_common.h"

int64_t pico_attn_bwd_split_workspace(const pico_attn_args* a);
int pico_attn_bwd_split(const pico_attn_args* a, hipStream_t s);

// Shared argument validation for forward and backward.
int pico_attn_check_common(const pico_attn_args* a, const char* op) {
  PICO_REQUIRE(a, "%s: null args", op);
  PICO_REQUIRE(a->q && a->k && a->v, "%s: null q/k/v", op);
  PICO_REQUIRE(a->head_dim == 64 || a->head_dim == 128, "%s: head_dim=%lld unsupported (64 or 128)", op,
               (long long)a->head_dim);
  PICO_REQUIRE(a->batch >= 0 && a->seqlen_q >= 0 && a->seqlen_k >= 0 && a->heads_q >= 0 && a->heads_kv > 0,
               "%s: bad sizes", op);
  PICO_REQUIRE(a->heads_q % a->heads_kv == 0, "%s: heads_q=%lld not a multiple of heads_kv=%lld", op,
               (long long)a->heads_q, (long long)a->heads_kv);
  PICO_REQUIRE(!a->causal || a->seqlen_q == a->seqlen_k, "%s: causal requires seqlen_q == seqlen_k", op);
  PICO_REQUIRE(a->seqlen_q < (1 << 30) && a->seqlen_k < (1 << 30), "%s: sequence too long", op);
  const int64_t* st[3] = {a->q_strides, a->k_strides, a->v_strides};
  for (int i = 0; i < 3; ++i)
    for (int d = 0; d < 3; ++d) PICO_REQUIRE(st[i][d] % 8 == 0, "%s: strides must be multiples of 8 elements", op);
  PICO_REQUIRE(((uintptr_t)a->q | (uintptr_t)a->k | (uintptr_t)a->v) % 16 == 0, "%s: q/k/v must be 16-byte aligned",
               op);
  return 0;
}

extern "C" {

int64_t pico_attn_args_size(void) { return (int64_t)sizeof(pico_attn_args); }

// [lse2 | delta] each [B*Hq][Sq padded to 32] fp32, + fp32 dK/dV partials when a small grid splits key blocks
int64_t pico_attn_bwd_workspace_bytes(const pico_attn_args* a) { return pico_attn_bwd_split_workspace(a); }

int pico_attn_bwd(const pico_attn_args* a, void* stream) {
  int rc = pico_attn_check_common(a, "pico_attn_bwd");
  if (rc) return rc;
  PICO_REQUIRE(a->o && a->lse && a->dout && a->dq && a->dk && a->dv && a->workspace, "pico_attn_bwd: null pointer");
  const int64_t* st[5] = {a->o_strides, a->do_strides, a->dq_strides, a->dk_strides, a->dv_strides};
  for (int i = 0; i < 5; ++i)
    for (int d = 0; d < 3; ++d)
      PICO_REQUIRE(st[i][d] % 8 == 0 || (i == 2 && (a->flags & PICO_ATTN_DQ_F32_ACCUM)),
                   "pico_attn_bwd: strides must be multiples of 8 elements");
  if (a->flags & PICO_ATTN_ROPE_BWD) {
    PICO_REQUIRE(!(a->flags & PICO_ATTN_DQ_F32_ACCUM), "pico_attn_bwd: ROPE_BWD cannot be combined with DQ_F32_ACCUM");
    PICO_REQUIRE(a->rope_cos && a->rope_sin && ((uintptr_t)a->rope_cos | (uintptr_t)a->rope_sin) % 16 == 0,
                 "pico_attn_bwd: ROPE_BWD needs 16-byte aligned cos/sin tables");
    PICO_REQUIRE(a->rope_stride % 8 == 0 && a->rope_stride >= a->head_dim / 2,
                 "pico_attn_bwd: bad rope table row stride %lld", (long long)a->rope_stride);
  }
  if (a->batch == 0 || a->seqlen_q == 0 || a->heads_q == 0) return 0;
  return pico_attn_bwd_split(a, (hipStream_t)stream);
}

}  // extern "C"
