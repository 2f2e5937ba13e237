// 2-D bf16 transpose for gfx950: dst[c][r] = src[r][c].
//
// Feeds the GEMM layouts hipBLASLt runs fastest on MI355X (scripts/gemm_layout_probe.py, M = 4096):
//   * wgrad dW = dy^T x accumulated into the gradient: with x^T contiguous the "TT" form
//     (dy^T (x^T)^T) beats the plain "TN" one (gate_up 263 -> 212 us, LM head 769 -> 643, qkv 107 -> 98),
//     so the fused projections keep x^T [K, T] instead of x for their backward;
//   * dgrad dx = dy W against a contiguous W^T (refreshed after each optimizer step).
// No reference counterpart: the reference leaves these layouts to cuBLAS (ref picotron/model.py
// nn.Linear). HBM-bound: 2 x rows x cols x 2 bytes per call.
//
// One 256-thread workgroup per 64 x 64 tile: 16-byte row loads (8 lanes per 128-byte row segment),
// tile staged in LDS with a 66-element row pitch, then each lane gathers 8 input rows of one column
// and stores them as one 16-byte segment of an output row (8 lanes per 128-byte output segment).
// LDS banks: the gather's dword address is (8 ch + i) * 33 + c / 2 -> banks 8 ch + c / 2 (mod 64),
// distinct over a wave (ch in 0..7, c / 2 in 0..3); the row writes hit 4 consecutive dwords per lane.
#include "common.h"

namespace {

constexpr int TT = 64;      // tile edge
constexpr int PITCH = 66;   // LDS row pitch in bf16 elements

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ src, int64_t ld_src,
                                                             bf16_t* __restrict__ dst, int64_t ld_dst, int64_t rows,
                                                             int64_t cols) {
  __shared__ unsigned short tile[TT * PITCH];
  const int64_t r0 = (int64_t)blockIdx.y * TT, c0 = (int64_t)blockIdx.x * TT;
  const int t = threadIdx.x;
  const int lr = t >> 3, lc = (t & 7) * 8;
  u16x8 v[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int64_t r = r0 + lr + 32 * p;
    if (r < rows && c0 + lc < cols) {
      v[p] = *reinterpret_cast<const u16x8*>(src + r * ld_src + c0 + lc);
    } else {
      v[p] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    unsigned* d = reinterpret_cast<unsigned*>(tile + (lr + 32 * p) * PITCH + lc);
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = (unsigned)v[p][2 * k] | ((unsigned)v[p][2 * k + 1] << 16);
  }
  __syncthreads();
  const int oc = t >> 3, ch = (t & 7) * 8;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int c = oc + 32 * p;
    u16x8 w;
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = tile[(ch + i) * PITCH + c];
    if (c0 + c < cols && r0 + ch < rows) *reinterpret_cast<u16x8*>(dst + (c0 + c) * ld_dst + r0 + ch) = w;
  }
}

}  // namespace

extern "C" int pico_transpose_bf16(const void* src, int64_t ld_src, void* dst, int64_t ld_dst, int64_t rows,
                                   int64_t cols, void* stream) {
  PICO_REQUIRE(rows >= 0 && cols >= 0, "pico_transpose_bf16: bad sizes");
  if (rows == 0 || cols == 0) return 0;
  PICO_REQUIRE(src && dst, "pico_transpose_bf16: null pointer");
  PICO_REQUIRE(rows % 8 == 0 && cols % 8 == 0, "pico_transpose_bf16: rows and cols must be multiples of 8");
  PICO_REQUIRE(ld_src >= cols && ld_dst >= rows && ld_src % 8 == 0 && ld_dst % 8 == 0,
               "pico_transpose_bf16: leading dims must cover the matrix and be multiples of 8");
  PICO_REQUIRE(((uintptr_t)src | (uintptr_t)dst) % 16 == 0, "pico_transpose_bf16: pointers must be 16-byte aligned");
  PICO_REQUIRE((rows + TT - 1) / TT <= 65535, "pico_transpose_bf16: too many rows");
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)pico_cdiv(cols, TT), (unsigned)pico_cdiv(rows, TT));
  PICO_TRY(pico_launch(PICO_K_TRANSPOSE, "transpose_bf16", transpose_bf16_kernel, dim3(grid), dim3(256), 0, s, (const bf16_t*)src, ld_src, (bf16_t*)dst, ld_dst, rows,
                                                         cols));
  return 0;
}
