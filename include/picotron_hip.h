/*
 * picotron_hip.h — C ABI of the MI355X (gfx950) hot-path kernels of picotron_amd.
 *
 * The reference (rkinas/picotron) is pure Python; its native arithmetic lives in
 * flash-attn 2.5.0 (CUDA + Triton) and torch ATen/NCCL. Each entry point below replaces one
 * of those third-party calls made from the reference's model / data-parallel code:
 *
 *   pico_rmsnorm_fwd / _bwd   <- flash_attn.ops.triton.layer_norm.layer_norm_fn(is_rms_norm=True)
 *                                 called by TritonRMSNorm.forward   (ref picotron/model.py:50-64)
 *                                 eager oracle LlamaRMSNorm          (ref picotron/model.py:66-85)
 *   pico_rope                 <- flash_attn.layers.rotary.apply_rotary_emb(x, cos, sin, interleaved=False)
 *                                 called by Attention.forward         (ref picotron/model.py:135-136)
 *                                 (conjugate=1 is its backward: rotation by -theta)
 *   pico_swiglu_fwd / _bwd    <- F.silu(gate(x)) * up(x)             (ref picotron/model.py:185)
 *   pico_attn_fwd / _bwd      <- flash_attn_func(q, k, v, causal)     (ref picotron/model.py:32-36,153)
 *                                 and the ring-attention block fwd/bwd
 *                                 (ref picotron/context_parallel/context_parallel.py:112-155)
 *   pico_attn_merge           <- update_out_and_lse                  (ref .../context_parallel.py:157-187)
 *   pico_grad_accum           <- param.main_grad.add_(param.grad)    (ref picotron/data_parallel/data_parallel.py:131)
 *                                 fused with Bucket.sync_gradient's grad_data /= W
 *                                                                      (ref picotron/data_parallel/bucket.py:30)
 *   pico_cast_f32_bf16        <- p.grad = p.main_grad.to(p.dtype)    (ref picotron/data_parallel/data_parallel.py:165)
 *   pico_scale_f32            <- grad_data /= process_group_size     (ref picotron/data_parallel/bucket.py:30)
 *   pico_cross_entropy_fwd/_bwd <- F.cross_entropy(logits, target, reduction='mean')
 *                                 (ref train.py:46-49, picotron/pipeline_parallel/pipeline_parallel.py:68,98)
 *   pico_adamw_bf16           <- torch.optim.AdamW(..., fused=True).step() (ref train.py:204-209,235)
 *   pico_sort_ids             <- the stable id sort inside F.embedding's backward (ref picotron/model.py:223-224)
 *   pico_embedding_bwd        <- backward of F.embedding (ref picotron/model.py:223-224) + the micro-batch
 *                                 gradient accumulation (data_parallel.py:131 / autograd's grad += dW)
 *   pico_transpose_bf16       <- no reference call: lays out x^T / W^T for the faster hipBLASLt forms of
 *                                 the nn.Linear wgrad / dgrad GEMMs (ref picotron/model.py nn.Linear)
 *
 * Conventions: all pointers are device pointers allocated by the caller (kernels never
 * allocate); bf16 tensors are passed as raw 16-bit storage; `stream` is a hipStream_t
 * (the caller's current stream). Every function returns 0 on success or a non-zero
 * status (hipError_t value, or PICO_EINVAL for argument errors); pico_last_error()
 * returns the message for the calling thread. No C++ exception crosses the ABI.
 */
#ifndef PICOTRON_HIP_H
#define PICOTRON_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PICO_ABI_VERSION 2
#define PICO_EINVAL 1000

/* kernel ids for the optional event timer (pico_prof_*) */
enum {
  PICO_K_RMSNORM_FWD = 1,
  PICO_K_RMSNORM_BWD = 2,
  PICO_K_RMSNORM_DW = 3,
  PICO_K_ROPE = 4,
  PICO_K_SWIGLU_FWD = 5,
  PICO_K_SWIGLU_BWD = 6,
  PICO_K_ATTN_FWD = 7,
  PICO_K_ATTN_BWD_PRE = 8, /* 8-10: retired with round 1's fused backward (kept so later ids stay stable) */
  PICO_K_ATTN_BWD = 9,
  PICO_K_ATTN_BWD_DQ = 10,
  PICO_K_GRAD_ACCUM = 11,
  PICO_K_CAST = 12,
  PICO_K_SCALE = 13,
  PICO_K_ATTN_MERGE = 14,
  PICO_K_EMBEDDING_BWD = 15,
  PICO_K_CE_FWD = 16,
  PICO_K_CE_BWD = 17,
  PICO_K_TRANSPOSE = 18,
  PICO_K_ATTN_BWD_DKV = 19,
  PICO_K_SORT_IDS = 20,
  PICO_K_ADAMW = 21,
  PICO_K_ATTN_BWD_KV = 22, /* split backward: dK/dV key-major kernel */
  PICO_K_ATTN_BWD_Q = 23,  /* split backward: dQ query-major kernel (+ delta, LSE*log2e) */
  PICO_K_COUNT = 24
};

int pico_abi_version(void);
const char* pico_last_error(void);

/* ---- event timer: times every launch of the enabled kernel ids on the stream each is launched on ----
 * pico_prof_enable(id, capacity) enables id (up to `capacity` timed launches); id <= 0 disables all.
 * pico_prof_collect(id, ...) synchronises the recorded events, returns their summed duration and
 * count, and resets that id's pool. */
int pico_prof_enable(int kernel_id, int capacity);
int pico_prof_collect(int kernel_id, double* total_ms, int64_t* launches);

/* ---- kernel selection (A/B switches; process-wide, read by every later launch) ----
 * Each knob starts at its shipped default (PICO_SEL_AUTO = the library's shape rule), overridden ONCE, when the
 * library is loaded, by the environment variable named beside it; pico_select(knob, value) sets it afterwards
 * (value PICO_SEL_AUTO restores the rule). Returns the previous value, or -2 for an unknown knob. No launch reads
 * the environment. */
#define PICO_SEL_AUTO (-1)
enum {
  PICO_SEL_ATTN_KVP = 0,    /* PICO_ATTN_KVP: dK/dV kernel, 1 = 64-row (attn_bwd_kvp_kernel at D=64,
                               attn_bwd_kvp128_kernel at D=128), 0 = 32-row kernel */
  PICO_SEL_KVP_WAVES = 1,   /* PICO_KVP_WAVES: waves per attn_bwd_kvp_kernel workgroup, 4 or 8 */
  PICO_SEL_ATTN_GROUPS = 2, /* PICO_ATTN_GROUPS: one-round block groups of the causal dK/dV grid, 1 on / 0 off */
  PICO_SEL_ATTN_FWD = 3,    /* PICO_ATTN_FWD: 1 = the persistent 64-row-per-wave forward (opt-in, measured slower) */
  PICO_SEL_COUNT = 4
};
int pico_select(int knob, int value);

/* ---- RMSNorm: y = x * rsqrt(mean(x^2) + eps) * w, fp32 math, one bf16 rounding ----
 * x, y: [rows, cols] bf16 row-major (row stride = cols); w: [cols] bf16; rstd: [rows] fp32 (saved
 * for backward). residual (optional, may be NULL): x_eff = bf16(x + residual), written to
 * residual_out when residual_out != NULL (layer_norm_fn(prenorm=True) semantics). */
/* pico_rmsnorm_fwd that also writes y^T ([cols, rows], row stride ld_t): the x^T the next projection's
 * weight-gradient GEMM reads. cols 1024 or 2048, rows multiple of 32, 16-byte aligned pointers. */
int pico_rmsnorm_fwd_t(const void* x, const void* residual, const void* weight, void* y, void* residual_out,
                       float* rstd, void* y_t, int64_t ld_t, int64_t rows, int64_t cols, float eps, void* stream);
int pico_rmsnorm_fwd(const void* x, const void* residual, const void* weight, void* y,
                     void* residual_out, float* rstd, int64_t rows, int64_t cols, float eps,
                     void* stream);
int64_t pico_rmsnorm_bwd_workspace_bytes(int64_t rows, int64_t cols);
/* dx: [rows, cols] bf16; dweight: [cols] bf16; workspace >= pico_rmsnorm_bwd_workspace_bytes.
 * dresidual (optional, may be NULL): added into dx (gradient flowing through residual_out). */
int pico_rmsnorm_bwd(const void* dy, const void* dresidual, const void* x, const void* weight,
                     const float* rstd, void* dx, void* dweight, void* workspace, int64_t rows,
                     int64_t cols, void* stream);
/* As pico_rmsnorm_bwd, with the weight gradient's micro-batch accumulation folded in (the
 * reference's AccumulateGrad `grad += dw` at DP = 1 / DataParallelBucket's `main_grad += grad`,
 * ref picotron/data_parallel/data_parallel.py:131, and the bucket's /W, bucket.py:30):
 *   dw_mode 0: dweight (bf16)  = sum                      (== pico_rmsnorm_bwd)
 *   dw_mode 1: dweight (bf16)  = bf16(dweight + sum)       (one rounding)
 *   dw_mode 2: dweight (fp32)  = (dweight + sum) * dw_scale */
int pico_rmsnorm_bwd_acc(const void* dy, const void* dresidual, const void* x, const void* weight,
                         const float* rstd, void* dx, void* dweight, int dw_mode, float dw_scale,
                         void* workspace, int64_t rows, int64_t cols, void* stream);
/* Chained form (one launch per norm instead of two): as pico_rmsnorm_bwd_acc, but
 *   reduce_own = 0 leaves this call's dw partial rows (pico_rmsnorm_bwd_partial_rows of them, [nb][cols]
 *     fp32) in `workspace` for a later call to reduce (dweight / dw_mode / dw_scale unused);
 *   prev_part != NULL: the same launch also reduces a previous call's partial rows ([prev_nb][prev_cols],
 *     still alive in the caller's memory) into prev_dweight with prev_mode / prev_scale.
 * pico_rmsnorm_dw_reduce does that reduction alone (the last norm of a backward pass). Deterministic: every
 * dw sum runs in a fixed order. */
int pico_rmsnorm_bwd_chain(const void* dy, const void* dresidual, const void* x, const void* weight,
                           const float* rstd, void* dx, void* dweight, int dw_mode, float dw_scale,
                           void* workspace, int64_t rows, int64_t cols, int reduce_own,
                           const float* prev_part, int64_t prev_nb, int64_t prev_cols, void* prev_dweight,
                           int prev_mode, float prev_scale, void* stream);
int64_t pico_rmsnorm_bwd_partial_rows(int64_t rows, int64_t cols);
int pico_rmsnorm_dw_reduce(const float* part, int64_t nb, int64_t cols, void* dweight, int dw_mode,
                           float dw_scale, void* stream);

/* ---- RoPE, rotate-half (non-interleaved) layout ----
 * x, out: [batch, seqlen, heads, head_dim] bf16 with element strides (batch, seq, head) and
 * unit last-dim stride (out may alias x). cos/sin: [seqlen, >= head_dim/2] bf16 tables with
 * row stride cs_stride (elements); element i < head_dim/2 of row s is cos(s * theta_i).
 * out[..., i]       = x[i] * c - x[i + D/2] * s
 * out[..., i + D/2] = x[i + D/2] * c + x[i] * s        (conjugate: s -> -s, the backward) */
int pico_rope(const void* x, void* out, const void* cos, const void* sin, int64_t batch,
              int64_t seqlen, int64_t heads, int64_t head_dim, const int64_t* x_strides,
              const int64_t* out_strides, int64_t cs_stride, int conjugate, void* stream);

/* ---- SwiGLU epilogue: h = silu(g) * u on [rows, cols] bf16 ----
 * gate/up (and dgate/dup) rows at element stride in_stride (they may be the two column halves of one
 * fused gate|up GEMM output, in_stride = 2*cols); out/dout rows at out_stride. */
/* pico_swiglu_fwd that also writes out^T ([cols, rows], row stride t_stride): the down projection's
 * x^T for its weight-gradient GEMM. rows, cols multiples of 64; strides multiples of 8. */
int pico_swiglu_fwd_t(const void* gate, const void* up, void* out, void* out_t, int64_t rows, int64_t cols,
                      int64_t in_stride, int64_t out_stride, int64_t t_stride, void* stream);
int pico_swiglu_fwd(const void* gate, const void* up, void* out, int64_t rows, int64_t cols,
                    int64_t in_stride, int64_t out_stride, void* stream);
int pico_swiglu_bwd(const void* dout, const void* gate, const void* up, void* dgate, void* dup,
                    int64_t rows, int64_t cols, int64_t in_stride, int64_t out_stride, void* stream);

/* ---- Flash attention (bf16 MFMA, online softmax, fp32 LSE) ----
 * Layouts: q/o/do/dq [B, Sq, Hq, D], k/v/dk/dv [B, Sk, Hkv, D] with element strides
 * (batch, seq, head) and unit last-dim stride; lse [B, Hq, Sq] fp32 contiguous (natural log,
 * lse = log sum_j exp(scale * q.k_j)). Hq % Hkv == 0 (GQA: query head h uses kv head h/(Hq/Hkv)).
 * head_dim in {64, 128}. causal requires Sq == Sk (top-left aligned mask j <= i). */
typedef struct pico_attn_args {
  const void* q;
  const void* k;
  const void* v;
  void* o;          /* fwd output / bwd input */
  float* lse;       /* fwd output / bwd input */
  const void* dout; /* bwd */
  void* dq;         /* bwd out (bf16, or fp32 accumulate with PICO_ATTN_DQ_F32_ACCUM) */
  void* dk;         /* bwd out bf16 */
  void* dv;         /* bwd out bf16 */
  void* workspace;  /* bwd: >= pico_attn_bwd_workspace_bytes */
  int64_t batch, seqlen_q, seqlen_k, heads_q, heads_kv, head_dim;
  int64_t q_strides[3], k_strides[3], v_strides[3], o_strides[3];
  int64_t do_strides[3], dq_strides[3], dk_strides[3], dv_strides[3];
  float softmax_scale;
  int causal;
  int flags;
  /* PICO_ATTN_ROPE_BWD: bf16 rotate-half tables [>= S, D/2] (row stride rope_stride elements) */
  const void* rope_cos;
  const void* rope_sin;
  int64_t rope_stride;
  /* fwd, optional (NULL: off): O also written transposed, o_t[hq * D + d][b * Sq + q] with row stride
   * o_t_ld elements — the [Hq*D, tokens] layout of the out-projection input that its weight-gradient
   * GEMM reads fastest (x^T), written from the accumulator layout at no extra pass */
  void* o_t;
  int64_t o_t_ld;
} pico_attn_args;

#define PICO_ATTN_DQ_F32_ACCUM 1 /* dq is fp32 [B,Sq,Hq,D] (dq_strides) and is ADDED into */
/* bwd: q and k were rotated (RoPE, rotate-half, position = sequence index) before attention; dq and dk
 * are returned rotated back by -theta (the RoPE backward, ref picotron/model.py:135-136), fused into
 * the dQ slab sum and the dK epilogue. Not combinable with PICO_ATTN_DQ_F32_ACCUM. */
#define PICO_ATTN_ROPE_BWD 2
/* fwd: q holds UNROTATED queries; each row is rotated (RoPE, rotate-half, position = sequence index,
 * tables as for ROPE_BWD) in registers before use, and the rotated rows are written to dq (dq_strides;
 * dq may alias q) for the backward. Replaces the query half of the separate pico_rope launch. */
#define PICO_ATTN_ROPE_Q_FWD 4

int64_t pico_attn_args_size(void); /* sizeof(pico_attn_args), for FFI layout checks */
int pico_attn_fwd(const pico_attn_args* args, void* stream);
int64_t pico_attn_bwd_workspace_bytes(const pico_attn_args* args);
int pico_attn_bwd(const pico_attn_args* args, void* stream);

/* ---- ring-attention block merge (update_out_and_lse) ----
 * ref picotron/context_parallel/context_parallel.py:157-187:
 *   first != 0: out = float(block_out), lse = block_lse
 *   otherwise:  out -= sigmoid(block_lse - lse) * (out - block_out); lse -= logsigmoid(lse - block_lse)
 * Every operand by element strides, so the reference's layout (out [B, H, S, D] fp32 and lse [B, H, S, 1],
 * or slices of them, ref :183-186) and the ring's internal [B, S, H, D] one use the same entry point:
 * out fp32, strides (batch, seq, head), unit head_dim stride; lse fp32, strides (batch, head, seq);
 * block_out bf16 (block_out_f32 == 0) or fp32, strides (batch, seq, head), unit head_dim stride;
 * block_lse fp32, strides (batch, head, seq). out and block_out rows 16-byte aligned. */
int pico_attn_merge(float* out, const int64_t* out_strides, float* lse, const int64_t* lse_strides,
                    const void* block_out, const int64_t* block_out_strides, int block_out_f32,
                    const float* block_lse, const int64_t* block_lse_strides, int64_t batch, int64_t seqlen,
                    int64_t heads, int64_t head_dim, int first, void* stream);

/* ---- DP gradient buckets ---- */
/* main_grad[i] = (main_grad[i] + float(grad[i])) * (1.0f / divide_by)   (divide_by == 1: no scaling).
 * The fp32 reciprocal product is what ATen computes for the reference's `grad_data /= W` on a GPU. */
int pico_grad_accum(float* main_grad, const void* grad, int64_t n, float divide_by, void* stream);
/* buf[i] = buf[i] * (1.0f / divide_by) */
int pico_scale_f32(float* buf, int64_t n, float divide_by, void* stream);
/* dst[i] = bf16(src[i]) (round to nearest even) */
int pico_cast_f32_bf16(const float* src, void* dst, int64_t n, void* stream);

/* ---- token embedding backward (deterministic, graph-safe) ----
 * sorted_ids / sorted_pos: the n_tokens token ids stable-sorted ascending and their positions
 * (int64, device). dy: [n_tokens, dim] bf16. grad: [vocab, dim] bf16 (grad_is_f32 = 0) or fp32;
 * for every id present: grad[id] = (grad[id] + sum of its dy rows in position order) * scale. */
int pico_embedding_bwd(const int64_t* sorted_ids, const int64_t* sorted_pos, const void* dy, void* grad,
                       int64_t n_tokens, int64_t dim, int grad_is_f32, float scale, void* stream);
/* Stable ascending sort of n <= 8192 token ids in [0, vocab), vocab <= 2^19 (int64, device) with their
 * positions: the input pico_embedding_bwd wants, bit-identical to torch.sort(ids, stable=True)
 * (which the reference's F.embedding backward does inside ATen). One workgroup, LDS bitonic sort of
 * (id << 13 | position) keys. */
int pico_sort_ids(const int64_t* ids, int64_t n, int64_t vocab, int64_t* sorted_ids, int64_t* sorted_pos,
                  void* stream);

/* ---- AdamW step over a whole parameter list (one launch) ----
 * Replaces torch.optim.AdamW(params, lr, fused=True).step() (ref train.py:13,204-209,235) for bf16
 * parameters with bf16 exp_avg / exp_avg_sq (torch keeps the states in the parameter dtype).
 * tensors: device int64 [n_tensors][5] = (param, grad, exp_avg, exp_avg_sq addresses, grad_is_f32);
 * grad_is_f32 != 0: grad is an fp32 buffer (DataParallelBucket's averaged main_grad with the bf16 .grad
 * cast deferred, ref picotron/data_parallel/data_parallel.py:165), rounded to bf16 in register exactly as
 * pico_cast_f32_bf16 stores it — bit-identical to cast-then-step; sizes: device int64 [n_tensors] numel; chunks: device int64 [n_chunks][2] = (tensor index, first element), one
 * per pico_adamw_chunk_elems() elements of each tensor. step: the step number after increment (>= 1).
 * Same expression order and types as ATen's fused AdamW (decoupled weight decay). */
int64_t pico_adamw_chunk_elems(void);
int pico_adamw_bf16(const int64_t* tensors, const int64_t* sizes, const int64_t* chunks, int64_t n_chunks,
                    double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step,
                    void* stream);

/* ---- softmax cross-entropy (mean over non-ignored rows) ----
 * logits: [rows, vocab] bf16, row stride ld (elements); target: [rows] int64.
 * fwd: lse[i] = log sum_j exp(logits[i][j]) (fp32), loss[i] = lse[i] - logits[i][target[i]] (0 for
 *      target == ignore_index). The caller sums loss[] and divides by the non-ignored count.
 * bwd: dlogits[i][j] = (exp(logits[i][j] - lse[i]) - [j == target[i]]) * (*grad_scale) (0 rows for
 *      ignored targets); grad_scale is a DEVICE fp32 scalar (grad_out / n_valid), row stride ldd. */
int pico_cross_entropy_fwd(const void* logits, int64_t ld, const int64_t* target, float* lse, float* loss,
                           int64_t rows, int64_t vocab, int64_t ignore_index, void* stream);
/* fused forward + gradient: as pico_cross_entropy_fwd, and the logits are overwritten IN PLACE with
 * (softmax - onehot) * (*grad_scale) (device fp32 scalar; 0 rows for ignored targets) — the gradient of
 * mean CE for a unit upstream gradient, which the caller scales after the LM-head GEMMs. */
int pico_cross_entropy_fwd_grad(void* logits, int64_t ld, const int64_t* target, float* lse, float* loss,
                                const float* grad_scale, int64_t rows, int64_t vocab, int64_t ignore_index,
                                void* stream);
/* The mean's scalars around pico_cross_entropy_fwd_grad, one launch each (instead of the ATen scalar ops of
 * F.cross_entropy(reduction='mean')'s host code): pico_ce_count writes stats[0] = #(target != ignore_index),
 * stats[1] = grad_scale / stats[0] (pass stats + 1 as fwd_grad's grad_scale); pico_ce_mean writes
 * grad_scale * sum(loss_rows) / stats[0] to *out (bf16, or fp32 when out_f32), summed in a fixed order,
 * and when acc is non-null adds the stored value to *acc (fp32): the training loop's per-step loss sum
 * (ref train.py:53 `loss_acc += loss.item()`), kept on the device without a separate launch. */
int pico_ce_count(const int64_t* target, int64_t n, int64_t ignore_index, float grad_scale, float* stats,
                  void* stream);
int pico_ce_mean(const float* loss_rows, int64_t n, const float* stats, float grad_scale, void* out, int out_f32,
                 float* acc, void* stream);
/* backward of the fused LM-head CE: dx (bf16, contiguous, n elements) *= *upstream (the loss's upstream
 * gradient, a device 0-dim bf16 tensor, or fp32 when upstream_f32, rounded to bf16 first as ATen does),
 * fp32 product, one bf16 rounding.
 * Replaces autograd's scaling of the reference's logits gradient (ref picotron/model.py:269, train.py:46-49).
 * nonunit (optional, device int): set to 1 if the upstream gradient is not exactly 1 (the chunked LM-head CE
 * accumulated its weight gradient in the forward for a unit upstream; the host checks the flag later). */
int pico_ce_scale_grad(void* dx, int64_t n, const void* upstream, int upstream_f32, int* nonunit, void* stream);
int pico_cross_entropy_bwd(const void* logits, int64_t ld, const int64_t* target, const float* lse,
                           const float* grad_scale, void* dlogits, int64_t ldd, int64_t rows, int64_t vocab,
                           int64_t ignore_index, void* stream);

/* ---- 2-D transpose ----
 * dst[c][r] = src[r][c] for a [rows, cols] bf16 matrix with row stride ld_src into [cols, rows] with row
 * stride ld_dst (elements). rows, cols, ld_src, ld_dst multiples of 8; pointers 16-byte aligned. */
int pico_transpose_bf16(const void* src, int64_t ld_src, void* dst, int64_t ld_dst, int64_t rows, int64_t cols,
                        void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PICOTRON_HIP_H */
