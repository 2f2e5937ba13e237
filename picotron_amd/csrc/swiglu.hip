// SwiGLU epilogue h = silu(g) * u, forward and backward (HBM-bound elementwise).
//
// Replaces the two ATen kernels of F.silu(self.gate_proj(x)) * self.up_proj(x)
// (ref picotron/model.py:183-185) and their autograd backward. fp32 math, one rounding per output.
// 8 bf16 per thread per tensor (16-byte loads/stores), grid-stride; gate and up may be the two
// column halves of one fused gate|up GEMM output (row stride 2*I), and the backward writes dgate/dup
// straight into the two halves of the fused GEMM's input gradient.
// Algorithmic bytes per element: fwd 3 * 2 B, bwd 5 * 2 B.
#include "common.h"

namespace {

PICO_DEV float sigmoidf_(float g) { return 1.f / (1.f + __expf(-g)); }

PICO_DEV void swiglu_grad(float dh, float gf, float uf, float& dg, float& du) {
  const float sg = sigmoidf_(gf);
  const float silu = gf * sg;
  du = dh * silu;
  dg = dh * uf * sg * (1.f + gf * (1.f - sg));
}

// 2-D strided form: gate/up rows of `cols` elements at row stride `in_stride` (gate and up may be
// the two column halves of one fused [rows, 2*cols] GEMM output), out rows at `out_stride`.
// Vector path: 8 elements (16 B) per thread; requires cols, strides % 8 == 0 and 16-B alignment.
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ u,
                                                         bf16_t* __restrict__ h, int64_t rows, int cols, int64_t is,
                                                         int64_t os) {
  const unsigned vpr = (unsigned)cols / 8;
  const unsigned nv = (unsigned)(rows * vpr);  // host guarantees < 2^31
  for (unsigned t = blockIdx.x * 256 + threadIdx.x; t < nv; t += gridDim.x * 256) {
    const unsigned row32 = t / vpr;
    const int64_t row = row32;
    const int c = (int)(t - row32 * vpr) * 8;
    const u16x8 gv = *reinterpret_cast<const u16x8*>(g + row * is + c);
    const u16x8 uv = *reinterpret_cast<const u16x8*>(u + row * is + c);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(gv[j]);
      o[j] = f2bf(gf * sigmoidf_(gf) * bf2f(uv[j]));
    }
    *reinterpret_cast<u16x8*>(h + row * os + c) = o;
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ dh, const bf16_t* __restrict__ g,
                                                         const bf16_t* __restrict__ u, bf16_t* __restrict__ dg,
                                                         bf16_t* __restrict__ du, int64_t rows, int cols, int64_t is,
                                                         int64_t os) {
  const unsigned vpr = (unsigned)cols / 8;
  const unsigned nv = (unsigned)(rows * vpr);  // host guarantees < 2^31
  for (unsigned t = blockIdx.x * 256 + threadIdx.x; t < nv; t += gridDim.x * 256) {
    const unsigned row32 = t / vpr;
    const int64_t row = row32;
    const int c = (int)(t - row32 * vpr) * 8;
    const u16x8 dv = *reinterpret_cast<const u16x8*>(dh + row * os + c);
    const u16x8 gv = *reinterpret_cast<const u16x8*>(g + row * is + c);
    const u16x8 uv = *reinterpret_cast<const u16x8*>(u + row * is + c);
    u16x8 og, ou;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a, b;
      swiglu_grad(bf2f(dv[j]), bf2f(gv[j]), bf2f(uv[j]), a, b);
      og[j] = f2bf(a);
      ou[j] = f2bf(b);
    }
    *reinterpret_cast<u16x8*>(dg + row * is + c) = og;
    *reinterpret_cast<u16x8*>(du + row * is + c) = ou;
  }
}

#ifndef PICO_SWIGLU_T_TC
#define PICO_SWIGLU_T_TC 128
#endif

// Forward that also writes h^T ([cols, rows], row stride ts) for the down projection's weight-gradient
// GEMM (its fast TT form reads x^T). One workgroup per 64 x TC tile (TC * 4 threads): 16-byte loads of
// the gate/up tile rows, h stored row-major, then the bf16 tile goes through LDS (TC + 2 element pitch,
// conflict-free column reads) and is stored as TC rows of h^T (128-B segments). TC = 128 by default
// (256-B row segments of g / u / h: 52.7 -> 48.5 us in-step against TC = 64; 256 measured the same as 128).
// Requires rows, cols multiple of 64 (host checks). Bytes: 3 * 2 B + 2 B (h^T) per element.
template <int TC>
__global__ __launch_bounds__(TC * 4) void swiglu_fwd_t_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ u,
                                                              bf16_t* __restrict__ h, bf16_t* __restrict__ ht, int64_t is,
                                                              int64_t os, int64_t ts) {
  constexpr int TP = TC + 2;  // LDS pitch (elements)
  __shared__ unsigned short tile[64 * TP];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * TC;
  const int t = threadIdx.x;
  const int lr = t / (TC / 8), lc = (t % (TC / 8)) * 8;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int64_t row = r0 + lr + 32 * p;
    const u16x8 gv = *reinterpret_cast<const u16x8*>(g + row * is + c0 + lc);
    const u16x8 uv = *reinterpret_cast<const u16x8*>(u + row * is + c0 + lc);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(gv[j]);
      o[j] = f2bf(gf * sigmoidf_(gf) * bf2f(uv[j]));
    }
    *reinterpret_cast<u16x8*>(h + row * os + c0 + lc) = o;
    unsigned* d = reinterpret_cast<unsigned*>(tile + (lr + 32 * p) * TP + lc);
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = (unsigned)o[2 * k] | ((unsigned)o[2 * k + 1] << 16);
  }
  __syncthreads();
  const int oc = t >> 3, ch = (t & 7) * 8;  // h^T row (a column of the tile), 8-token chunk
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int c = oc + (TC / 2) * p;
    u16x8 w;
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = tile[(ch + i) * TP + c];
    *reinterpret_cast<u16x8*>(ht + (c0 + c) * ts + r0 + ch) = w;
  }
}

// scalar fallback (unaligned / ragged shapes)
__global__ __launch_bounds__(256) void swiglu_fwd_scalar(const bf16_t* __restrict__ g, const bf16_t* __restrict__ u,
                                                         bf16_t* __restrict__ h, int64_t rows, int cols, int64_t is,
                                                         int64_t os) {
  const int64_t n = rows * cols;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const int64_t row = t / cols;
    const int c = (int)(t - row * cols);
    const float gf = bf2f(g[row * is + c]);
    h[row * os + c] = f2bf(gf * sigmoidf_(gf) * bf2f(u[row * is + c]));
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_scalar(const bf16_t* __restrict__ dh, const bf16_t* __restrict__ g,
                                                         const bf16_t* __restrict__ u, bf16_t* __restrict__ dg,
                                                         bf16_t* __restrict__ du, int64_t rows, int cols, int64_t is,
                                                         int64_t os) {
  const int64_t n = rows * cols;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += (int64_t)gridDim.x * 256) {
    const int64_t row = t / cols;
    const int c = (int)(t - row * cols);
    float a, b;
    swiglu_grad(bf2f(dh[row * os + c]), bf2f(g[row * is + c]), bf2f(u[row * is + c]), a, b);
    dg[row * is + c] = f2bf(a);
    du[row * is + c] = f2bf(b);
  }
}

int grid_for(int64_t work) {
  int64_t nb = (work + 255) / 256;
  if (nb < 1) nb = 1;
  if (nb > 4096) nb = 4096;  // 256 CUs x 16 workgroups, grid-stride beyond
  return (int)nb;
}

bool vec_ok(int64_t cols, int64_t is, int64_t os, const void* a, const void* b, const void* c) {
  return cols % 8 == 0 && is % 8 == 0 && os % 8 == 0 && ((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) % 16 == 0;
}

}  // namespace

extern "C" {

int pico_swiglu_fwd_t(const void* gate, const void* up, void* out, void* out_t, int64_t rows, int64_t cols,
                      int64_t in_stride, int64_t out_stride, int64_t t_stride, void* stream) {
  PICO_REQUIRE(gate && up && out && out_t, "pico_swiglu_fwd_t: null pointer");
  PICO_REQUIRE(rows >= 0 && cols >= 0 && rows % 64 == 0 && cols % 64 == 0,
               "pico_swiglu_fwd_t: rows and cols must be multiples of 64");
  PICO_REQUIRE(in_stride >= cols && out_stride >= cols && t_stride >= rows && in_stride % 8 == 0 &&
                   out_stride % 8 == 0 && t_stride % 8 == 0,
               "pico_swiglu_fwd_t: strides must cover the matrix and be multiples of 8");
  PICO_REQUIRE((((uintptr_t)gate | (uintptr_t)up | (uintptr_t)out | (uintptr_t)out_t) & 15) == 0,
               "pico_swiglu_fwd_t: pointers must be 16-byte aligned");
  PICO_REQUIRE(rows / 64 <= 65535, "pico_swiglu_fwd_t: too many rows");
  if (rows == 0 || cols == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (PICO_SWIGLU_T_TC == 256 && cols % 256 == 0) {
    PICO_TRY(pico_launch(PICO_K_SWIGLU_FWD, "swiglu_fwd_t", swiglu_fwd_t_kernel<256>, dim3((unsigned)(cols / 256), (unsigned)(rows / 64)),
                         dim3(1024), 0, s, (const bf16_t*)gate, (const bf16_t*)up, (bf16_t*)out, (bf16_t*)out_t, in_stride,
                         out_stride, t_stride));
  } else if (PICO_SWIGLU_T_TC >= 128 && cols % 128 == 0) {
    PICO_TRY(pico_launch(PICO_K_SWIGLU_FWD, "swiglu_fwd_t", swiglu_fwd_t_kernel<128>, dim3((unsigned)(cols / 128), (unsigned)(rows / 64)),
                         dim3(512), 0, s, (const bf16_t*)gate, (const bf16_t*)up, (bf16_t*)out, (bf16_t*)out_t, in_stride,
                         out_stride, t_stride));
  } else {
    PICO_TRY(pico_launch(PICO_K_SWIGLU_FWD, "swiglu_fwd_t", swiglu_fwd_t_kernel<64>, dim3((unsigned)(cols / 64), (unsigned)(rows / 64)),
                         dim3(256), 0, s, (const bf16_t*)gate, (const bf16_t*)up, (bf16_t*)out, (bf16_t*)out_t, in_stride,
                         out_stride, t_stride));
  }
  return 0;
}

int pico_swiglu_fwd(const void* gate, const void* up, void* out, int64_t rows, int64_t cols, int64_t in_stride,
                    int64_t out_stride, void* stream) {
  PICO_REQUIRE(gate && up && out, "pico_swiglu_fwd: null pointer");
  PICO_REQUIRE(rows >= 0 && cols >= 0 && cols < (1ll << 31) && in_stride >= cols && out_stride >= cols,
               "pico_swiglu_fwd: bad shape");
  if (rows * cols == 0) return 0;
  PICO_REQUIRE(rows * cols < (1ll << 31), "pico_swiglu_fwd: tensor too large");
  hipStream_t s = (hipStream_t)stream;
  auto g = (const bf16_t*)gate;
  auto u = (const bf16_t*)up;
  auto h = (bf16_t*)out;
  if (vec_ok(cols, in_stride, out_stride, gate, up, out)) {
    PICO_TRY(pico_launch(PICO_K_SWIGLU_FWD, "swiglu_fwd", swiglu_fwd_kernel, dim3(grid_for(rows * cols / 8)), dim3(256), 0, s, g, u, h, rows, (int)cols, in_stride,
                                                                             out_stride));
  } else {
    PICO_TRY(pico_launch(PICO_K_SWIGLU_FWD, "swiglu_fwd", swiglu_fwd_scalar, dim3(grid_for(rows * cols)), dim3(256), 0, s, g, u, h, rows, (int)cols, in_stride,
                                                                        out_stride));
  }
  return 0;
}

int pico_swiglu_bwd(const void* dout, const void* gate, const void* up, void* dgate, void* dup, int64_t rows,
                    int64_t cols, int64_t in_stride, int64_t out_stride, void* stream) {
  PICO_REQUIRE(dout && gate && up && dgate && dup, "pico_swiglu_bwd: null pointer");
  PICO_REQUIRE(rows >= 0 && cols >= 0 && cols < (1ll << 31) && in_stride >= cols && out_stride >= cols,
               "pico_swiglu_bwd: bad shape");
  if (rows * cols == 0) return 0;
  PICO_REQUIRE(rows * cols < (1ll << 31), "pico_swiglu_bwd: tensor too large");
  hipStream_t s = (hipStream_t)stream;
  const bool vec = vec_ok(cols, in_stride, out_stride, dout, gate, up) &&
                   ((uintptr_t)dgate | (uintptr_t)dup) % 16 == 0;
  if (vec) {
    PICO_TRY(pico_launch(PICO_K_SWIGLU_BWD, "swiglu_bwd", swiglu_bwd_kernel, dim3(grid_for(rows * cols / 8)), dim3(256), 0, s, (const bf16_t*)dout, (const bf16_t*)gate, (const bf16_t*)up, (bf16_t*)dgate, (bf16_t*)dup, rows,
                    (int)cols, in_stride, out_stride));
  } else {
    PICO_TRY(pico_launch(PICO_K_SWIGLU_BWD, "swiglu_bwd", swiglu_bwd_scalar, dim3(grid_for(rows * cols)), dim3(256), 0, s, (const bf16_t*)dout, (const bf16_t*)gate, (const bf16_t*)up, (bf16_t*)dgate, (bf16_t*)dup, rows,
                    (int)cols, in_stride, out_stride));
  }
  return 0;
}

}  // extern "C"
