// Fused softmax cross-entropy over the LM-head logits for gfx950 (HBM-bound).
//
// Replaces F.cross_entropy(logits, target, reduction='mean') (ref train.py:46-49,
// picotron/pipeline_parallel/pipeline_parallel.py:68,98). ATen runs it as log_softmax -> nll_loss
// and back (nll_loss backward materialises a dense one-hot gradient, log_softmax backward re-reads
// it and the saved log-probabilities): about six sweeps over the [tokens, vocab] logits (SmolLM:
// 4096 x 49152 bf16 = 403 MB each). Here:
//   fwd: one read of the logits -> per-row lse (fp32) and loss_i = lse_i - x_i[t_i];
//   bwd: one read of the logits -> dlogits = (exp(x - lse) - onehot(t)) * grad_out / n_valid, written
//        once (bf16), with grad_out / n_valid read from device memory (no host sync).
// Rows whose target == ignore_index contribute neither loss nor gradient (torch semantics).
// One 256-thread workgroup per row; a thread keeps its NCH 16-byte chunks of the row in registers
// between the max and the sum-of-exp passes, so each pass reads the row from HBM once.
// fp32 math throughout (torch: fp32 opmath inside log_softmax, bf16 log-probs in between).
#include "common.h"

// PICO_CE_THREADS: threads per logits row in the fused forward+gradient kernel (A/B build variants)
#ifndef PICO_CE_THREADS
#define PICO_CE_THREADS 512
#endif
constexpr float LOG2E = 1.4426950408889634f;

namespace {

PICO_DEV float wave_max_dpp(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false)));
  const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r16[0]), __uint_as_float(r16[1]));
  const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r32[0]), __uint_as_float(r32[1]));
}

template <int NT>
PICO_DEV float block_reduce(float v, float* red, bool is_max) {
  v = is_max ? wave_max_dpp(v) : wave_sum_dpp(v);  // DPP / permlane, no LDS round trips
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int k = 1; k < NT / 64; ++k) r = is_max ? fmaxf(r, red[k]) : r + red[k];
  return r;
}

template <int NCH>
__global__ __launch_bounds__(256) void ce_fwd_kernel(const bf16_t* __restrict__ logits, int64_t ld,
                                                     const int64_t* __restrict__ target, float* __restrict__ lse,
                                                     float* __restrict__ loss, int vocab, int64_t ignore) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  const bf16_t* x = logits + row * ld;
  const int nchunk = vocab / 8;
  u16x8 v[NCH];
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = threadIdx.x + 256 * c;
    if (ch < nchunk) {
      v[c] = *reinterpret_cast<const u16x8*>(x + 8 * ch);
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, bf2f(v[c][j]));
    }
  }
  m = block_reduce<256>(m, red, true);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = threadIdx.x + 256 * c;
    if (ch < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __builtin_amdgcn_exp2f((bf2f(v[c][j]) - m) * 1.4426950408889634f);
    }
  }
  s = block_reduce<256>(s, red, false);
  if (threadIdx.x == 0) {
    const float l = m + __logf(s);
    const int64_t t = target[row];
    lse[row] = l;
    loss[row] = (t == ignore || t < 0 || t >= vocab) ? 0.f : l - bf2f(x[t]);
  }
}

template <int NCH>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const bf16_t* __restrict__ logits, int64_t ld,
                                                     const int64_t* __restrict__ target, const float* __restrict__ lse,
                                                     const float* __restrict__ gscale, bf16_t* __restrict__ dlogits,
                                                     int64_t ldd, int vocab, int64_t ignore) {
  const int64_t row = blockIdx.x;
  const bf16_t* x = logits + row * ld;
  bf16_t* dx = dlogits + row * ldd;
  const int nchunk = vocab / 8;
  const int64_t t = target[row];
  const bool skip = t == ignore || t < 0 || t >= vocab;
  const float g = skip ? 0.f : *gscale;
  const float l = lse[row];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = threadIdx.x + 256 * c;
    if (ch < nchunk) {
      const u16x8 xv = *reinterpret_cast<const u16x8*>(x + 8 * ch);
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float p = __expf(bf2f(xv[j]) - l);
        if (8 * ch + j == t) p -= 1.f;
        o[j] = f2bf(p * g);
      }
      *reinterpret_cast<u16x8*>(dx + 8 * ch) = o;
    }
  }
}

// Forward that also produces the gradient in place: lse, loss as ce_fwd_kernel, then the row (still in
// registers) is overwritten with dlogits = (softmax - onehot(t)) * (*gscale) (0 for ignored rows). One
// read + one write of the logits instead of fwd read + bwd read + bwd write; the caller applies the
// upstream gradient later (it scales the LM-head GEMMs' results, not the logits).
template <int NCH, int NT>
__global__ __launch_bounds__(NT) void ce_fwd_grad_kernel(bf16_t* __restrict__ logits, int64_t ld,
                                                          const int64_t* __restrict__ target, float* __restrict__ lse,
                                                          float* __restrict__ loss, const float* __restrict__ gscale,
                                                          int vocab, int64_t ignore) {
  __shared__ float red[NT / 64];
  const int64_t row = blockIdx.x;
  bf16_t* x = logits + row * ld;
  const int nchunk = vocab / 8;
  const int64_t t = target[row];
  const bool skip = t == ignore || t < 0 || t >= vocab;
  const float xt = skip ? 0.f : bf2f(x[skip ? 0 : t]);  // read before the row is overwritten
  u16x8 v[NCH];
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = threadIdx.x + NT * c;
    if (ch < nchunk) {
      v[c] = *reinterpret_cast<const u16x8*>(x + 8 * ch);
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, bf2f(v[c][j]));
    }
  }
  m = block_reduce<NT>(m, red, true);
  float s = 0.f;
  const float nm2 = -m * LOG2E;  // exp(x - m) = exp2(fma(x, log2 e, -m log2 e)): one FMA per logit
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = threadIdx.x + NT * c;
    if (ch < nchunk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __builtin_amdgcn_exp2f(__builtin_fmaf(bf2f(v[c][j]), LOG2E, nm2));
    }
  }
  s = block_reduce<NT>(s, red, false);
  const float l = m + __logf(s);
  if (threadIdx.x == 0) {
    lse[row] = l;
    loss[row] = skip ? 0.f : l - xt;
  }
  const float g = skip ? 0.f : *gscale;
  // softmax * g = exp2(x log2 e - l log2 e + log2 g): one FMA + one exp2 per logit (g = 0 -> log2 g =
  // -inf -> 0 for ignored rows); the one-hot term is applied afterwards by the lane that owns the
  // target (its later store to the same address wins)
  const float c2 = __builtin_fmaf(-l, LOG2E, __log2f(g));
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int ch = threadIdx.x + NT * c;
    if (ch < nchunk) {
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(__builtin_amdgcn_exp2f(__builtin_fmaf(bf2f(v[c][j]), LOG2E, c2)));
      *reinterpret_cast<u16x8*>(x + 8 * ch) = o;
    }
  }
  if (!skip && (int)(t >> 3) % NT == (int)threadIdx.x) {
    const float pt = __builtin_amdgcn_exp2f(__builtin_fmaf(xt, LOG2E, c2));
    x[t] = f2bf(pt - g);
  }
}

int nch_for(int64_t vocab, int nt = 256) {
  const int64_t per = (vocab / 8 + nt - 1) / nt;
  for (int n : {2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64})
    if (per <= n) return n;
  return -1;
}

}  // namespace

#define CE_SWITCH(NCHV, CALL)                      \
  switch (NCHV) {                                  \
    case 2: { constexpr int N = 2; CALL; } break;   \
    case 3: { constexpr int N = 3; CALL; } break;   \
    case 6: { constexpr int N = 6; CALL; } break;   \
    case 12: { constexpr int N = 12; CALL; } break; \
    case 4: { constexpr int N = 4; CALL; } break;   \
    case 8: { constexpr int N = 8; CALL; } break;   \
    case 16: { constexpr int N = 16; CALL; } break; \
    case 24: { constexpr int N = 24; CALL; } break; \
    case 32: { constexpr int N = 32; CALL; } break; \
    case 48: { constexpr int N = 48; CALL; } break; \
    case 64: { constexpr int N = 64; CALL; } break; \
  }

extern "C" int pico_cross_entropy_fwd(const void* logits, int64_t ld, const int64_t* target, float* lse, float* loss,
                                      int64_t rows, int64_t vocab, int64_t ignore_index, void* stream) {
  PICO_REQUIRE(rows >= 0 && vocab > 0 && vocab % 8 == 0 && ld % 8 == 0 && ld >= vocab,
               "pico_cross_entropy_fwd: vocab (%lld) and row stride must be multiples of 8", (long long)vocab);
  const int nch = nch_for(vocab);
  PICO_REQUIRE(nch > 0, "pico_cross_entropy_fwd: vocab %lld too large", (long long)vocab);
  PICO_REQUIRE(rows < (1ll << 31), "pico_cross_entropy_fwd: too many rows");
  if (rows == 0) return 0;
  PICO_REQUIRE(logits && target && lse && loss, "pico_cross_entropy_fwd: null pointer");
  hipStream_t s = (hipStream_t)stream;
  CE_SWITCH(nch, PICO_TRY(pico_launch(PICO_K_CE_FWD, "cross_entropy_fwd", ce_fwd_kernel<N>, dim3((int)rows), dim3(256), 0, s, (const bf16_t*)logits, ld, target, lse, loss,
                                                                        (int)vocab, ignore_index)))
  return 0;
}

extern "C" int pico_cross_entropy_fwd_grad(void* logits, int64_t ld, const int64_t* target, float* lse, float* loss,
                                           const float* grad_scale, int64_t rows, int64_t vocab, int64_t ignore_index,
                                           void* stream) {
  PICO_REQUIRE(rows >= 0 && vocab > 0 && vocab % 8 == 0 && ld % 8 == 0 && ld >= vocab,
               "pico_cross_entropy_fwd_grad: vocab (%lld) and row stride must be multiples of 8", (long long)vocab);
  const int nch = nch_for(vocab, PICO_CE_THREADS);
  PICO_REQUIRE(nch > 0, "pico_cross_entropy_fwd_grad: vocab %lld too large", (long long)vocab);
  PICO_REQUIRE(rows < (1ll << 31), "pico_cross_entropy_fwd_grad: too many rows");
  if (rows == 0) return 0;
  PICO_REQUIRE(logits && target && lse && loss && grad_scale, "pico_cross_entropy_fwd_grad: null pointer");
  hipStream_t s = (hipStream_t)stream;
  CE_SWITCH(nch, PICO_TRY(pico_launch(PICO_K_CE_FWD, "cross_entropy_fwd_grad", ce_fwd_grad_kernel<N, PICO_CE_THREADS>, dim3((int)rows), dim3(PICO_CE_THREADS), 0, s, (bf16_t*)logits, ld, target, lse, loss,
                                                                             grad_scale, (int)vocab, ignore_index)))
  return 0;
}

extern "C" int pico_cross_entropy_bwd(const void* logits, int64_t ld, const int64_t* target, const float* lse,
                                      const float* grad_scale, void* dlogits, int64_t ldd, int64_t rows, int64_t vocab,
                                      int64_t ignore_index, void* stream) {
  PICO_REQUIRE(rows >= 0 && vocab > 0 && vocab % 8 == 0 && ld % 8 == 0 && ldd % 8 == 0,
               "pico_cross_entropy_bwd: vocab and row strides must be multiples of 8");
  const int nch = nch_for(vocab);
  PICO_REQUIRE(nch > 0, "pico_cross_entropy_bwd: vocab %lld too large", (long long)vocab);
  if (rows == 0) return 0;
  PICO_REQUIRE(logits && target && lse && grad_scale && dlogits, "pico_cross_entropy_bwd: null pointer");
  hipStream_t s = (hipStream_t)stream;
  CE_SWITCH(nch, PICO_TRY(pico_launch(PICO_K_CE_BWD, "cross_entropy_bwd", ce_bwd_kernel<N>, dim3((int)rows), dim3(256), 0, s, (const bf16_t*)logits, ld, target, lse,
                                                                        grad_scale, (bf16_t*)dlogits, ldd, (int)vocab,
                                                                        ignore_index)))
  return 0;
}

// ---------------------------------------------------------------------------------------------------
// The mean's scalar bookkeeping around the fused LM-head CE (ref train.py:46-49, reduction='mean'), one
// 1024-thread workgroup each instead of ~9 ATen scalar launches per micro-batch:
//   pico_ce_count: stats[0] = number of targets != ignore_index, stats[1] = grad_scale / stats[0]
//     (the per-row gradient scale pico_cross_entropy_fwd_grad reads);
//   pico_ce_mean: out (bf16, or fp32 when out_f32) = grad_scale * sum(loss_rows) / stats[0],
//     summed in a fixed order (deterministic); acc (optional, fp32) += that value as stored in out — the
//     training loop's per-step loss sum (`loss_acc += loss`, ref train.py:53) without a separate launch.
namespace {
constexpr int CE_NT = 1024;

PICO_DEV float block_sum_1024(float v, float* red) {
  v = wave_sum_dpp(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0)
    for (int w = 0; w < CE_NT / 64; ++w) t += red[w];  // waves in order
  return t;
}

__global__ __launch_bounds__(CE_NT) void ce_count_kernel(const int64_t* __restrict__ target, int64_t n,
                                                         int64_t ignore_index, float grad_scale, float* stats) {
  __shared__ float red[CE_NT / 64];
  float c = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += CE_NT) c += target[i] != ignore_index ? 1.f : 0.f;
  const float t = block_sum_1024(c, red);  // exact: integer counts below 2^24
  if (threadIdx.x == 0) {
    stats[0] = t;
    stats[1] = grad_scale / t;
  }
}

__global__ __launch_bounds__(CE_NT) void ce_mean_kernel(const float* __restrict__ loss_rows, int64_t n,
                                                        const float* __restrict__ stats, float grad_scale, void* out,
                                                        int out_f32, float* acc) {
  __shared__ float red[CE_NT / 64];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n; i += CE_NT) s += loss_rows[i];
  const float t = block_sum_1024(s, red);
  if (threadIdx.x == 0) {
    float v = t / stats[0] * grad_scale;
    if (out_f32) {
      *(float*)out = v;
    } else {
      const bf16_t b = f2bf(v);
      *(bf16_t*)out = b;
      v = bf2f(b);
    }
    if (acc) *acc += v;
  }
}
}  // namespace

extern "C" int pico_ce_count(const int64_t* target, int64_t n, int64_t ignore_index, float grad_scale, float* stats,
                             void* stream) {
  PICO_REQUIRE(target && stats && n >= 0, "pico_ce_count: bad arguments");
  PICO_TRY(pico_launch(PICO_K_CE_FWD, "ce_count", ce_count_kernel, dim3(1), dim3(CE_NT), 0, (hipStream_t)stream, target, n, ignore_index, grad_scale, stats));
  return 0;
}

extern "C" int pico_ce_mean(const float* loss_rows, int64_t n, const float* stats, float grad_scale, void* out,
                            int out_f32, float* acc, void* stream) {
  PICO_REQUIRE(loss_rows && stats && out && n >= 0, "pico_ce_mean: bad arguments");
  PICO_TRY(pico_launch(PICO_K_CE_FWD, "ce_mean", ce_mean_kernel, dim3(1), dim3(CE_NT), 0, (hipStream_t)stream, loss_rows, n, stats, grad_scale, out, out_f32, acc));
  return 0;
}

// ---------------------------------------------------------------------------------------------------
// The fused LM-head CE's backward: dx (bf16, contiguous, computed in the forward for a unit upstream
// gradient) *= the upstream gradient, read from the device (bf16 or fp32 0-dim tensor) — the same
// rounding as ATen's bf16 tensor * 0-dim tensor (the 0-dim operand cast to bf16 first, then an fp32
// product and one bf16 rounding), without the
// broadcasting elementwise kernel that op lowers to (≈ 33 us per micro-batch at 4096 x 2048; this one
// streams 16-byte vectors). nonunit (optional): set to 1 when the upstream gradient is not exactly 1 — the
// chunked LM-head CE took its weight gradient in the forward for a unit upstream, and the host reports a
// violation the next time it reads this flag (no synchronisation here).
namespace {
__global__ __launch_bounds__(256) void scale_by_dev_kernel(bf16_t* __restrict__ x, int64_t n,
                                                           const void* __restrict__ g, int g_f32, int* nonunit) {
  const float graw = g_f32 ? *(const float*)g : bf2f(*(const bf16_t*)g);
  const float s = bf2f(g_f32 ? f2bf(graw) : *(const bf16_t*)g);
  if (nonunit && blockIdx.x == 0 && threadIdx.x == 0 && graw != 1.f) *nonunit = 1;
  const int64_t nv = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (int64_t)gridDim.x * 256) {
    u16x8 v = reinterpret_cast<u16x8*>(x)[i];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = f2bf(bf2f(v[j]) * s);
    reinterpret_cast<u16x8*>(x)[i] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x < (int)(n - 8 * nv)) x[8 * nv + threadIdx.x] = f2bf(bf2f(x[8 * nv + threadIdx.x]) * s);
}
}  // namespace

extern "C" int pico_ce_scale_grad(void* dx, int64_t n, const void* upstream, int upstream_f32, int* nonunit,
                                  void* stream) {
  PICO_REQUIRE(dx && upstream && n >= 0, "pico_ce_scale_grad: bad arguments");
  PICO_REQUIRE((uintptr_t)dx % 16 == 0, "pico_ce_scale_grad: dx must be 16-byte aligned");
  if (n == 0) return 0;
  int64_t nb = (n / 8 + 255) / 256;
  if (nb < 1) nb = 1;
  if (nb > 4096) nb = 4096;
  PICO_TRY(pico_launch(PICO_K_CE_BWD, "ce_scale_grad", scale_by_dev_kernel, dim3((int)nb), dim3(256), 0, (hipStream_t)stream, (bf16_t*)dx, n, upstream, upstream_f32, nonunit));
  return 0;
}
