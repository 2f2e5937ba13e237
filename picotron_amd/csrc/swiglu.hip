// SwiGLU epilogue h = silu(g) * u, forward and backward (HBM-bound elementwise).
//
// Replaces the two ATen kernels of F.silu(self.gate_proj(x)) * self.up_proj(x)
// (ref picotron/model.py:183-185) and their autograd backward. fp32 math, one rounding per output.
// 8 bf16 per thread per tensor (16-byte loads/stores), grid-stride.
// Algorithmic bytes per element: fwd 3 * 2 B, bwd 5 * 2 B.
#include "common.h"

namespace {

PICO_DEV float sigmoidf_(float g) { return 1.f / (1.f + __expf(-g)); }

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ u,
                                                         bf16_t* __restrict__ h, int64_t n) {
  const int64_t nv = n / 8;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < nv; t += stride) {
    const u16x8 gv = reinterpret_cast<const u16x8*>(g)[t];
    const u16x8 uv = reinterpret_cast<const u16x8*>(u)[t];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(gv[j]);
      o[j] = f2bf(gf * sigmoidf_(gf) * bf2f(uv[j]));
    }
    reinterpret_cast<u16x8*>(h)[t] = o;
  }
  // scalar tail (n % 8 elements), handled by the first threads of block 0
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
    const int64_t i = nv * 8 + threadIdx.x;
    const float gf = bf2f(g[i]);
    h[i] = f2bf(gf * sigmoidf_(gf) * bf2f(u[i]));
  }
}

PICO_DEV void swiglu_grad(float dh, float gf, float uf, float& dg, float& du) {
  const float sg = sigmoidf_(gf);
  const float silu = gf * sg;
  du = dh * silu;
  dg = dh * uf * sg * (1.f + gf * (1.f - sg));
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ dh, const bf16_t* __restrict__ g,
                                                         const bf16_t* __restrict__ u, bf16_t* __restrict__ dg,
                                                         bf16_t* __restrict__ du, int64_t n) {
  const int64_t nv = n / 8;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < nv; t += stride) {
    const u16x8 dv = reinterpret_cast<const u16x8*>(dh)[t];
    const u16x8 gv = reinterpret_cast<const u16x8*>(g)[t];
    const u16x8 uv = reinterpret_cast<const u16x8*>(u)[t];
    u16x8 og, ou;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a, b;
      swiglu_grad(bf2f(dv[j]), bf2f(gv[j]), bf2f(uv[j]), a, b);
      og[j] = f2bf(a);
      ou[j] = f2bf(b);
    }
    reinterpret_cast<u16x8*>(dg)[t] = og;
    reinterpret_cast<u16x8*>(du)[t] = ou;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
    const int64_t i = nv * 8 + threadIdx.x;
    float a, b;
    swiglu_grad(bf2f(dh[i]), bf2f(g[i]), bf2f(u[i]), a, b);
    dg[i] = f2bf(a);
    du[i] = f2bf(b);
  }
}

int grid_for(int64_t n) {
  int64_t nb = (n / 8 + 255) / 256;
  if (nb < 1) nb = 1;
  if (nb > 4096) nb = 4096;  // 256 CUs x 16 workgroups, grid-stride beyond
  return (int)nb;
}

}  // namespace

extern "C" {

int pico_swiglu_fwd(const void* gate, const void* up, void* out, int64_t n, void* stream) {
  PICO_REQUIRE(gate && up && out, "pico_swiglu_fwd: null pointer");
  PICO_REQUIRE(((uintptr_t)gate | (uintptr_t)up | (uintptr_t)out) % 16 == 0,
               "pico_swiglu_fwd: pointers must be 16-byte aligned");
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  PICO_LAUNCH(PICO_K_SWIGLU_FWD, "swiglu_fwd", s,
              swiglu_fwd_kernel<<<grid_for(n), 256, 0, s>>>((const bf16_t*)gate, (const bf16_t*)up, (bf16_t*)out, n));
  return 0;
}

int pico_swiglu_bwd(const void* dout, const void* gate, const void* up, void* dgate, void* dup, int64_t n,
                    void* stream) {
  PICO_REQUIRE(dout && gate && up && dgate && dup, "pico_swiglu_bwd: null pointer");
  PICO_REQUIRE(((uintptr_t)dout | (uintptr_t)gate | (uintptr_t)up | (uintptr_t)dgate | (uintptr_t)dup) % 16 == 0,
               "pico_swiglu_bwd: pointers must be 16-byte aligned");
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  PICO_LAUNCH(PICO_K_SWIGLU_BWD, "swiglu_bwd", s,
              swiglu_bwd_kernel<<<grid_for(n), 256, 0, s>>>((const bf16_t*)dout, (const bf16_t*)gate,
                                                            (const bf16_t*)up, (bf16_t*)dgate, (bf16_t*)dup, n));
  return 0;
}

}  // extern "C"
