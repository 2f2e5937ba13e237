// Fused RMSNorm forward/backward for gfx950 (HBM-bound).
//
// Replaces flash-attn's Triton layer_norm_fn(is_rms_norm=True) used by TritonRMSNorm
// (ref picotron/model.py:38-64). Math follows the reference's fused path: the row statistic and
// the product with the weight are done in fp32 and rounded to bf16 once
// (the eager oracle LlamaRMSNorm, ref picotron/model.py:80-85, rounds x_hat to bf16 before
// multiplying by w; the difference is within one bf16 ulp and covered by the parity tolerance).
//
// Layout: one wave64 per row, 4 rows per 256-thread workgroup; a lane owns 8 contiguous bf16
// per 512-column chunk (16-byte loads), and keeps the whole row in registers (MAXC chunks) so x
// is read from HBM exactly once. Algorithmic bytes: fwd 2*cols*2 B + 4 B per row,
// bwd 3*cols*2 B + 4 B per row (+ the small fp32 dw partials).
#include "common.h"

namespace {

constexpr int WAVES = 4;

PICO_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

PICO_DEV void load8(const bf16_t* p, float* f) {
  u16x8 v = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = bf2f(v[j]);
}

PICO_DEV void store8(bf16_t* p, const float* f) {
  u16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(f[j]);
  *reinterpret_cast<u16x8*>(p) = v;
}

template <int MAXC>
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                          const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                                          bf16_t* __restrict__ res_out, float* __restrict__ rstd,
                                                          int64_t rows, int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16_t* xr = x + row * cols;
  float v[MAXC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < cols) {
      load8(xr + col, v[c]);
      if (res) {
        float r[8];
        load8(res + row * cols + col, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = bf2f(f2bf(v[c][j] + r[j]));
        if (res_out) store8(res_out + row * cols + col, v[c]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
    }
  }
  ss = wave_sum(ss);
  const float rs = rsqrtf(ss / (float)cols + eps);
  if (lane == 0) rstd[row] = rs;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < cols) {
      float wf[8], o[8];
      load8(w + col, wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[c][j] * rs * wf[j];
      store8(y + row * cols + col, o);
    }
  }
}

// Backward: dx = rstd * (g - xhat * mean(g * xhat)), g = dy * w, xhat = x * rstd;
// dw partial per workgroup (deterministic two-stage reduction, no atomics).
template <int MAXC>
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ dres,
                                                          const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                          const float* __restrict__ rstd, bf16_t* __restrict__ dx,
                                                          float* __restrict__ dw_part, int64_t rows, int cols) {
  __shared__ float red[WAVES][MAXC * 512];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  float wf[MAXC][8], dwacc[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int col = (c * 64 + lane) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) dwacc[c][j] = 0.f;
    if (col < cols) load8(w + col, wf[c]);
  }
  for (int64_t row = (int64_t)blockIdx.x * WAVES + wid; row < rows; row += (int64_t)gridDim.x * WAVES) {
    const float rs = rstd[row];
    float xh[MAXC][8], g[MAXC][8];
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (col < cols) {
        float d[8];
        load8(x + row * cols + col, xh[c]);
        load8(dy + row * cols + col, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[c][j] *= rs;
          g[c][j] = d[j] * wf[c][j];
          dwacc[c][j] += d[j] * xh[c][j];
          dot += g[c][j] * xh[c][j];
        }
      }
    }
    dot = wave_sum(dot) / (float)cols;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (col < cols) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rs * (g[c][j] - xh[c][j] * dot);
        if (dres) {
          float r[8];
          load8(dres + row * cols + col, r);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += r[j];
        }
        store8(dx + row * cols + col, o);
      }
    }
  }
  // reduce the 4 waves' dw partials through LDS, write one fp32 row per workgroup
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wid][(c * 64 + lane) * 8 + j] = dwacc[c][j];
  __syncthreads();
  for (int col = threadIdx.x; col < cols; col += 256) {
    float s = red[0][col] + red[1][col] + red[2][col] + red[3][col];
    dw_part[(int64_t)blockIdx.x * cols + col] = s;
  }
}

// dw[col] = sum over the workgroup partials, in a fixed order (deterministic): a 256-thread
// workgroup covers 32 columns x 8 row-slices; each thread sums its slice (loads coalesced across the
// 32 columns), then the 8 slices are combined through LDS in slice order.
__global__ __launch_bounds__(256) void rmsnorm_dw_kernel(const float* __restrict__ part, bf16_t* __restrict__ dw, int nblk,
                                                         int cols) {
  __shared__ float red[8][32];
  const int c = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int col = blockIdx.x * 32 + c;
  float s = 0.f;
  if (col < cols) {
#pragma unroll 8
    for (int b = sl; b < nblk; b += 8) s += part[(int64_t)b * cols + col];
  }
  red[sl][c] = s;
  __syncthreads();
  if (sl == 0 && col < cols) {
    float t = red[0][c];
#pragma unroll
    for (int k = 1; k < 8; ++k) t += red[k][c];
    dw[col] = f2bf(t);
  }
}

int maxc_for(int64_t cols) {
  int64_t c = (cols + 511) / 512;
  if (c <= 1) return 1;
  if (c <= 2) return 2;
  if (c <= 4) return 4;
  if (c <= 8) return 8;
  if (c <= 16) return 16;
  return -1;
}

int bwd_blocks(int64_t rows) {  // one workgroup per CU at most: fewer dw partial rows to reduce
  int64_t nb = (rows + WAVES - 1) / WAVES;
  return (int)(nb < 256 ? nb : 256);
}

}  // namespace

extern "C" {

int pico_rmsnorm_fwd(const void* x, const void* residual, const void* weight, void* y, void* residual_out,
                     float* rstd, int64_t rows, int64_t cols, float eps, void* stream) {
  PICO_REQUIRE(x && weight && y && rstd, "pico_rmsnorm_fwd: null pointer");
  PICO_REQUIRE(rows >= 0 && cols > 0 && cols % 8 == 0, "pico_rmsnorm_fwd: cols=%lld must be a positive multiple of 8",
               (long long)cols);
  const int mc = maxc_for(cols);
  PICO_REQUIRE(mc > 0, "pico_rmsnorm_fwd: cols=%lld > 8192 unsupported", (long long)cols);
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(pico_cdiv(rows, WAVES)), block(256);
  auto xp = (const bf16_t*)x;
  auto rp = (const bf16_t*)residual;
  auto wp = (const bf16_t*)weight;
  auto yp = (bf16_t*)y;
  auto rop = (bf16_t*)residual_out;
  const int c = (int)cols;
#define FWD_CASE(M) \
  case M:           \
    PICO_LAUNCH(PICO_K_RMSNORM_FWD, "rmsnorm_fwd", s, rmsnorm_fwd_kernel<M><<<grid, block, 0, s>>>(xp, rp, wp, yp, rop, rstd, rows, c, eps)); \
    break;
  switch (mc) {
    FWD_CASE(1) FWD_CASE(2) FWD_CASE(4) FWD_CASE(8) FWD_CASE(16)
  }
#undef FWD_CASE
  return 0;
}

int64_t pico_rmsnorm_bwd_workspace_bytes(int64_t rows, int64_t cols) {
  return (int64_t)bwd_blocks(rows) * cols * (int64_t)sizeof(float);
}

int pico_rmsnorm_bwd(const void* dy, const void* dresidual, const void* x, const void* weight, const float* rstd,
                     void* dx, void* dweight, void* workspace, int64_t rows, int64_t cols, void* stream) {
  PICO_REQUIRE(dy && x && weight && rstd && dx && dweight && workspace, "pico_rmsnorm_bwd: null pointer");
  PICO_REQUIRE(rows > 0 && cols > 0 && cols % 8 == 0, "pico_rmsnorm_bwd: bad shape rows=%lld cols=%lld",
               (long long)rows, (long long)cols);
  const int mc = maxc_for(cols);
  PICO_REQUIRE(mc > 0 && mc <= 8, "pico_rmsnorm_bwd: cols=%lld > 4096 unsupported", (long long)cols);
  hipStream_t s = (hipStream_t)stream;
  const int nb = bwd_blocks(rows);
  auto part = (float*)workspace;
  const int c = (int)cols;
#define BWD_CASE(M)                                                                                          \
  case M:                                                                                                    \
    PICO_LAUNCH(PICO_K_RMSNORM_BWD, "rmsnorm_bwd", s,                                                        \
                rmsnorm_bwd_kernel<M><<<nb, 256, 0, s>>>((const bf16_t*)dy, (const bf16_t*)dresidual,       \
                                                         (const bf16_t*)x, (const bf16_t*)weight, rstd,      \
                                                         (bf16_t*)dx, part, rows, c));                      \
    break;
  switch (mc) {
    BWD_CASE(1) BWD_CASE(2) BWD_CASE(4) BWD_CASE(8)
  }
#undef BWD_CASE
  PICO_LAUNCH(PICO_K_RMSNORM_DW, "rmsnorm_dw", s,
              rmsnorm_dw_kernel<<<pico_cdiv(cols, 32), 256, 0, s>>>(part, (bf16_t*)dweight, nb, c));
  return 0;
}

}  // extern "C"
