// Token-embedding backward for gfx950, deterministic and HIP-graph safe.
//
// Replaces the backward of F.embedding(x, weight) (ref picotron/model.py:223-224) plus the
// micro-batch accumulation of its gradient (AccumulateGrad's `grad += dW` at DP = 1, or
// DataParallelBucket's `main_grad += grad`, ref picotron/data_parallel/data_parallel.py:131).
// ATen's dense backward materialises a [V, H] gradient that is almost all zeros (SmolLM: 100 M
// elements = 200 MB written, then 600 MB for the accumulate) and sizes its unique/partition work
// on the host, which a graph replay cannot redo. Here the caller stable-sorts the token ids
// (torch.sort, device-only), and one workgroup per sorted position that starts a run of equal ids
// sums that run's dy rows in position order (fp32) and updates only that id's row in place:
//   grad[id] = (grad[id] + sum) * scale        (bf16 or fp32 gradient; one rounding)
// Every row is owned by exactly one workgroup (no atomics); the summation order is fixed.
// Bytes: dy read once (T * H * 2) + touched rows read and written once.
#include "common.h"

namespace {

template <bool F32>
__global__ __launch_bounds__(256) void embedding_bwd_kernel(const int64_t* __restrict__ sorted_ids,
                                                            const int64_t* __restrict__ sorted_pos,
                                                            const bf16_t* __restrict__ dy, void* __restrict__ grad,
                                                            int64_t n, int64_t dim, float scale) {
  const int64_t b = blockIdx.x;
  const int64_t id = sorted_ids[b];
  if (b > 0 && sorted_ids[b - 1] == id) return;  // not the start of a run
  for (int64_t c = (int64_t)threadIdx.x * 8; c < dim; c += 256 * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int64_t j = b; j < n && sorted_ids[j] == id; ++j) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(dy + sorted_pos[j] * dim + c);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += bf2f(v[k]);
    }
    if constexpr (F32) {
      f32x4* g = reinterpret_cast<f32x4*>((float*)grad + id * dim + c);
      f32x4 a = g[0], bb = g[1];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[k] = (a[k] + acc[k]) * scale;
        bb[k] = (bb[k] + acc[4 + k]) * scale;
      }
      g[0] = a;
      g[1] = bb;
    } else {
      u16x8* g = reinterpret_cast<u16x8*>((bf16_t*)grad + id * dim + c);
      u16x8 w = *g;
#pragma unroll
      for (int k = 0; k < 8; ++k) w[k] = f2bf((bf2f(w[k]) + acc[k]) * scale);
      *g = w;
    }
  }
}

}  // namespace

extern "C" int pico_embedding_bwd(const int64_t* sorted_ids, const int64_t* sorted_pos, const void* dy, void* grad,
                                  int64_t n_tokens, int64_t dim, int grad_is_f32, float scale, void* stream) {
  PICO_REQUIRE(n_tokens >= 0 && dim > 0, "pico_embedding_bwd: bad sizes");
  PICO_REQUIRE(dim % 8 == 0, "pico_embedding_bwd: dim must be a multiple of 8");
  PICO_REQUIRE(n_tokens < (1ll << 31), "pico_embedding_bwd: too many tokens");
  if (n_tokens == 0) return 0;
  PICO_REQUIRE(sorted_ids && sorted_pos && dy && grad, "pico_embedding_bwd: null pointer");
  PICO_REQUIRE(((uintptr_t)dy | (uintptr_t)grad) % 16 == 0, "pico_embedding_bwd: dy/grad must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  if (grad_is_f32) {
    PICO_LAUNCH(PICO_K_EMBEDDING_BWD, "embedding_bwd", s,
                embedding_bwd_kernel<true><<<(int)n_tokens, 256, 0, s>>>(sorted_ids, sorted_pos, (const bf16_t*)dy,
                                                                         grad, n_tokens, dim, scale));
  } else {
    PICO_LAUNCH(PICO_K_EMBEDDING_BWD, "embedding_bwd", s,
                embedding_bwd_kernel<false><<<(int)n_tokens, 256, 0, s>>>(sorted_ids, sorted_pos, (const bf16_t*)dy,
                                                                          grad, n_tokens, dim, scale));
  }
  return 0;
}
