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
//
// pico_sort_ids replaces the torch.sort(ids, stable=True) in front of it (ATen: index copies, an
// arange and a 64-bit key/value radix sort, ~60 us at 4096 tokens): one 1024-thread workgroup
// bitonic-sorts 32-bit keys (id << 13 | position) in LDS, three stages per barrier. Positions are unique, so the order of equal
// ids is their position order (the stable order), and the result is bit-identical to torch's.
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

constexpr int SORT_POS_BITS = 13;  // positions < 8192
constexpr int SORT_MAX = 1 << SORT_POS_BITS;

// one pad word per 32 keys: the strided group loads of the small strides spread over the banks
__device__ __forceinline__ int pad(int i) { return i + (i >> 5); }

// M consecutive bitonic stages (strides jlo << (M-1) .. jlo) of merge size k in registers: each thread
// loads groups of 2^M keys closed under those stages, so one barrier covers M stages.
template <int M>
__device__ __forceinline__ void bitonic_pass(unsigned* key, int p2, int k, int jlo) {
  constexpr int G = 1 << M;
  for (int g = threadIdx.x; g < (p2 >> M); g += 1024) {
    const int base = ((g & ~(jlo - 1)) << M) | (g & (jlo - 1));
    const bool up = (base & k) == 0;
    unsigned v[G];
#pragma unroll
    for (int t = 0; t < G; ++t) v[t] = key[pad(base + t * jlo)];
#pragma unroll
    for (int s = M - 1; s >= 0; --s)
#pragma unroll
      for (int t = 0; t < G; ++t)
        if (!(t & (1 << s))) {
          const unsigned x = v[t], y = v[t | (1 << s)];
          const bool sw = (x > y) == up;
          v[t] = sw ? y : x;
          v[t | (1 << s)] = sw ? x : y;
        }
#pragma unroll
    for (int t = 0; t < G; ++t) key[pad(base + t * jlo)] = v[t];
  }
}

__global__ __launch_bounds__(1024) void sort_ids_kernel(const int64_t* __restrict__ ids, int n, int p2,
                                                        int64_t* __restrict__ sorted_ids,
                                                        int64_t* __restrict__ sorted_pos) {
  __shared__ unsigned key[SORT_MAX + SORT_MAX / 32];
  for (int i = threadIdx.x; i < p2; i += 1024)
    key[pad(i)] = i < n ? ((unsigned)ids[i] << SORT_POS_BITS) | (unsigned)i : 0xFFFFFFFFu;
  __syncthreads();
  for (int k = 2; k <= p2; k <<= 1) {
    for (int j = k >> 1; j > 0;) {
      const int m = min(3, 32 - __clz(j));  // stages left at this k: log2(j) + 1
      const int jlo = j >> (m - 1);
      if (m == 3) bitonic_pass<3>(key, p2, k, jlo);
      else if (m == 2) bitonic_pass<2>(key, p2, k, jlo);
      else bitonic_pass<1>(key, p2, k, jlo);
      __syncthreads();
      j = jlo >> 1;
    }
  }
  for (int i = threadIdx.x; i < n; i += 1024) {
    const unsigned v = key[pad(i)];
    sorted_ids[i] = (int64_t)(v >> SORT_POS_BITS);
    sorted_pos[i] = (int64_t)(v & (SORT_MAX - 1));
  }
}

}  // namespace

extern "C" int pico_sort_ids(const int64_t* ids, int64_t n, int64_t vocab, int64_t* sorted_ids, int64_t* sorted_pos,
                             void* stream) {
  PICO_REQUIRE(n >= 0 && n <= SORT_MAX, "pico_sort_ids: n (%lld) must be <= %d", (long long)n, SORT_MAX);
  PICO_REQUIRE(vocab > 0 && vocab <= (1ll << (32 - SORT_POS_BITS)), "pico_sort_ids: vocab (%lld) must be <= 2^19",
               (long long)vocab);
  if (n == 0) return 0;
  PICO_REQUIRE(ids && sorted_ids && sorted_pos, "pico_sort_ids: null pointer");
  int p2 = 2;
  while (p2 < n) p2 <<= 1;
  hipStream_t s = (hipStream_t)stream;
  PICO_TRY(pico_launch(PICO_K_SORT_IDS, "sort_ids", sort_ids_kernel, dim3(1), dim3(1024), 0, s, ids, (int)n, p2, sorted_ids, sorted_pos));
  return 0;
}

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
    PICO_TRY(pico_launch(PICO_K_EMBEDDING_BWD, "embedding_bwd", embedding_bwd_kernel<true>, dim3((int)n_tokens), dim3(256), 0, s, sorted_ids, sorted_pos, (const bf16_t*)dy,
                                                                         grad, n_tokens, dim, scale));
  } else {
    PICO_TRY(pico_launch(PICO_K_EMBEDDING_BWD, "embedding_bwd", embedding_bwd_kernel<false>, dim3((int)n_tokens), dim3(256), 0, s, sorted_ids, sorted_pos, (const bf16_t*)dy,
                                                                          grad, n_tokens, dim, scale));
  }
  return 0;
}
