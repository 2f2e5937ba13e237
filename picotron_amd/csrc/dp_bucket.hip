// Data-parallel gradient-bucket kernels (HBM-bound, bit-exact with the reference's ATen ops).
//
// pico_grad_accum    : main_grad += grad (fp32 += bf16), ref picotron/data_parallel/data_parallel.py:131.
//                      On the syncing micro-batch the bucket pre-scale grad_data /= W
//                      (ref picotron/data_parallel/bucket.py:30) is folded in. On the GPU, ATen evaluates
//                      `tensor /= python_scalar` as tensor * fp32(1/W) (its scalar-divisor fast path), so
//                      (m + g) * fp32(1/W) is the same two correctly-rounded fp32 ops as the reference's
//                      add_ followed by /=: bit-identical, with the bucket read and written once.
// pico_scale_f32     : grad_data /= W for buckets whose params were accumulated unscaled.
// pico_cast_f32_bf16 : p.grad = p.main_grad.to(bf16) (ref data_parallel.py:165), one launch per bucket.
//
// Bytes per element: accumulate 4+2+4 = 10 B, scale 8 B, cast 4+2 = 6 B.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void grad_accum_vec(float* __restrict__ m, const bf16_t* __restrict__ g, int64_t nv,
                                                      float inv, int do_div) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < nv; t += stride) {
    const u16x8 gv = reinterpret_cast<const u16x8*>(g)[t];
    f32x4 a = reinterpret_cast<const f32x4*>(m)[2 * t];
    f32x4 b = reinterpret_cast<const f32x4*>(m)[2 * t + 1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] = a[j] + bf2f(gv[j]);
      b[j] = b[j] + bf2f(gv[4 + j]);
      if (do_div) {
        a[j] = a[j] * inv;
        b[j] = b[j] * inv;
      }
    }
    reinterpret_cast<f32x4*>(m)[2 * t] = a;
    reinterpret_cast<f32x4*>(m)[2 * t + 1] = b;
  }
}

__global__ __launch_bounds__(256) void grad_accum_scalar(float* __restrict__ m, const bf16_t* __restrict__ g, int64_t n,
                                                         float inv, int do_div) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    float v = m[i] + bf2f(g[i]);
    if (do_div) v = v * inv;
    m[i] = v;
  }
}

__global__ __launch_bounds__(256) void scale_kernel(float* __restrict__ m, int64_t n, float inv) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t nv = n / 4;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < nv; t += stride) {
    f32x4 a = reinterpret_cast<const f32x4*>(m)[t];
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = a[j] * inv;
    reinterpret_cast<f32x4*>(m)[t] = a;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = nv * 4 + threadIdx.x;
    m[i] = m[i] * inv;
  }
}

__global__ __launch_bounds__(256) void cast_vec(const float* __restrict__ src, bf16_t* __restrict__ dst, int64_t nv) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < nv; t += stride) {
    const f32x4 a = reinterpret_cast<const f32x4*>(src)[2 * t];
    const f32x4 b = reinterpret_cast<const f32x4*>(src)[2 * t + 1];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = f2bf(a[j]);
      o[4 + j] = f2bf(b[j]);
    }
    reinterpret_cast<u16x8*>(dst)[t] = o;
  }
}

__global__ __launch_bounds__(256) void cast_scalar(const float* __restrict__ src, bf16_t* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) dst[i] = f2bf(src[i]);
}

int grid_for(int64_t work) {
  int64_t nb = (work + 255) / 256;
  if (nb < 1) nb = 1;
  if (nb > 4096) nb = 4096;
  return (int)nb;
}

}  // namespace

extern "C" {

int pico_grad_accum(float* main_grad, const void* grad, int64_t n, float divide_by, void* stream) {
  PICO_REQUIRE(main_grad && grad, "pico_grad_accum: null pointer");
  PICO_REQUIRE(divide_by > 0.f, "pico_grad_accum: divide_by must be > 0");
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int do_div = divide_by != 1.f;
  const float inv = 1.f / divide_by;  // fp32 reciprocal, as ATen's scalar-divisor path computes it
  const bool vec = n % 8 == 0 && (uintptr_t)main_grad % 32 == 0 && (uintptr_t)grad % 16 == 0;
  if (vec) {
    PICO_TRY(pico_launch(PICO_K_GRAD_ACCUM, "grad_accum", grad_accum_vec, dim3(grid_for(n / 8)), dim3(256), 0, s, main_grad, (const bf16_t*)grad, n / 8, inv, do_div));
  } else {
    PICO_TRY(pico_launch(PICO_K_GRAD_ACCUM, "grad_accum", grad_accum_scalar, dim3(grid_for(n)), dim3(256), 0, s, main_grad, (const bf16_t*)grad, n, inv, do_div));
  }
  return 0;
}

int pico_scale_f32(float* buf, int64_t n, float divide_by, void* stream) {
  PICO_REQUIRE(buf, "pico_scale_f32: null pointer");
  PICO_REQUIRE(divide_by > 0.f, "pico_scale_f32: divide_by must be > 0");
  PICO_REQUIRE((uintptr_t)buf % 16 == 0, "pico_scale_f32: buffer must be 16-byte aligned");
  if (n <= 0 || divide_by == 1.f) return 0;
  hipStream_t s = (hipStream_t)stream;
  PICO_TRY(pico_launch(PICO_K_SCALE, "scale_f32", scale_kernel, dim3(grid_for(n / 4)), dim3(256), 0, s, buf, n, 1.f / divide_by));
  return 0;
}

int pico_cast_f32_bf16(const float* src, void* dst, int64_t n, void* stream) {
  PICO_REQUIRE(src && dst, "pico_cast_f32_bf16: null pointer");
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const bool vec = n % 8 == 0 && (uintptr_t)src % 32 == 0 && (uintptr_t)dst % 16 == 0;
  if (vec) {
    PICO_TRY(pico_launch(PICO_K_CAST, "cast_f32_bf16", cast_vec, dim3(grid_for(n / 8)), dim3(256), 0, s, src, (bf16_t*)dst, n / 8));
  } else {
    PICO_TRY(pico_launch(PICO_K_CAST, "cast_f32_bf16", cast_scalar, dim3(grid_for(n)), dim3(256), 0, s, src, (bf16_t*)dst, n));
  }
  return 0;
}

}  // extern "C"
