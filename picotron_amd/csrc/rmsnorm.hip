// Fused RMSNorm forward/backward for gfx950 (HBM-bound).
//
// Replaces flash-attn's Triton layer_norm_fn(is_rms_norm=True) used by TritonRMSNorm
// (ref picotron/model.py:38-64). Math follows the reference's fused path: the row statistic and
// the product with the weight are done in fp32 and rounded to bf16 once
// (the eager oracle LlamaRMSNorm, ref picotron/model.py:80-85, rounds x_hat to bf16 before
// multiplying by w; the difference is within one bf16 ulp and covered by the parity tolerance).
//
// Layout (fwd): one wave64 per row, 4 rows per 256-thread workgroup; a lane owns 8 contiguous bf16
// per 512-column chunk (16-byte loads), and keeps the whole row in registers (MAXC chunks) so x
// is read from HBM exactly once. Algorithmic bytes: fwd 2*cols*2 B + 4 B per row,
// bwd 3*cols*2 B + 4 B per row (+ the small fp32 dw partials).
#include "common.h"

namespace {

constexpr int WAVES = 4;

PICO_DEV float wave_sum(float v) { return wave_sum_dpp(v); }

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

// Forward that also writes y^T ([cols, rows], row stride ldt): the x^T the following projection's
// weight-gradient GEMM reads (TT form), at the cost of one extra write instead of a transpose pass.
// One 512-thread workgroup per 32 rows (wave w: rows w, w + 8, ...; a lane owns 8 contiguous columns
// per 512-column chunk as in rmsnorm_fwd_kernel); y is also staged into an LDS tile [32][cols + 8]
// (128.5 KiB at cols = 2048), then each thread stores 8-token segments of y^T rows (4 x 16 B per
// 64-B row segment). Requires cols == MAXC * 512 and rows % 32 == 0 (host checks).
#ifndef PICO_RMS_FWDT_WAVES
#define PICO_RMS_FWDT_WAVES 8
#endif
// rows per tile: 32 (128 workgroups at 4096 rows: half the CUs) or 16 (256 workgroups); with 16, the two
// tiles whose y^T segments share each 64-byte line run on one XCD (blocks b and b + 8), so its L2 can merge
// the two 32-byte halves before they reach HBM
#ifndef PICO_RMS_FWDT_ROWS
#define PICO_RMS_FWDT_ROWS 16
#endif
#ifndef PICO_RMS_FWDT_QUAD
#define PICO_RMS_FWDT_QUAD 1
#endif
constexpr int FWDT_WAVES = PICO_RMS_FWDT_WAVES;  // waves per tile (rows per wave = FWDT_ROWS / FWDT_WAVES)
constexpr int FWDT_ROWS = PICO_RMS_FWDT_ROWS;
static_assert(FWDT_ROWS == 16 || FWDT_ROWS == 32, "tile rows");

template <int MAXC, bool RES>
__global__ __launch_bounds__(FWDT_WAVES * 64) void rmsnorm_fwd_t_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                            const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                                            bf16_t* __restrict__ res_out, float* __restrict__ rstd,
                                                            bf16_t* __restrict__ yt, int64_t ldt, float eps) {
  constexpr int COLS = MAXC * 512, PITCH = COLS + 8;
  extern __shared__ __attribute__((aligned(16))) unsigned short tile[];  // [FWDT_ROWS][PITCH]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t tidx = blockIdx.x;
  if (FWDT_ROWS == 16 && PICO_RMS_FWDT_QUAD && (gridDim.x & 31) == 0) {
    // blocks b, b + 8, b + 16, b + 24 (one XCD): the four tiles (4p .. 4p + 3) whose 32-byte y^T segments
    // make one 128-byte line
    const int64_t b = blockIdx.x, g = b >> 5;
    const int xcd = (int)(b & 7), q = (int)((b >> 3) & 3);
    tidx = 4 * (g * 8 + xcd) + q;
  } else if (FWDT_ROWS == 16 && (gridDim.x & 15) == 0) {  // blocks b, b + 8 (one XCD): tile pair (2p, 2p + 1)
    const int64_t b = blockIdx.x, g = b >> 4;
    const int xcd = (int)(b & 7), half = (int)((b >> 3) & 1);
    tidx = 2 * (g * 8 + xcd) + half;
  }
  const int64_t r0 = tidx * FWDT_ROWS;
  constexpr int RPW = FWDT_ROWS / FWDT_WAVES;  // rows per wave (rows wid + FWDT_WAVES k): every load issued first
  u16x8 xr[RPW][MAXC], rr[RPW][MAXC];
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int64_t row = r0 + wid + FWDT_WAVES * k;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int col = (c * 64 + lane) * 8;
      xr[k][c] = *reinterpret_cast<const u16x8*>(x + row * COLS + col);
      if constexpr (RES) rr[k][c] = *reinterpret_cast<const u16x8*>(res + row * COLS + col);
    }
  }
  float ss[RPW];
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int64_t row = r0 + wid + FWDT_WAVES * k;
    ss[k] = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int col = (c * 64 + lane) * 8;
      if constexpr (RES) {
        u16x8 sum;
#pragma unroll
        for (int j = 0; j < 8; ++j) sum[j] = f2bf(bf2f(xr[k][c][j]) + bf2f(rr[k][c][j]));
        xr[k][c] = sum;
        if (res_out) *reinterpret_cast<u16x8*>(res_out + row * COLS + col) = sum;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = bf2f(xr[k][c][j]);
        ss[k] += v * v;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < RPW; ++k) ss[k] = wave_sum(ss[k]);
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int lr = wid + FWDT_WAVES * k;
    const int64_t row = r0 + lr;
    const float rs = rsqrtf(ss[k] / (float)COLS + eps);
    if (lane == 0) rstd[row] = rs;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int col = (c * 64 + lane) * 8;
      float wf[8];
      load8(w + col, wf);
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(xr[k][c][j]) * rs * wf[j]);
      *reinterpret_cast<u16x8*>(y + row * COLS + col) = o;
      *reinterpret_cast<u16x8*>(tile + lr * PITCH + col) = o;
    }
  }
  __syncthreads();
  // a task = 2 adjacent columns x 8 tokens: 8 dword LDS reads -> two 16-byte y^T segments
  constexpr int NPART = FWDT_ROWS / 8;
  for (int task = threadIdx.x; task < COLS / 2 * NPART; task += FWDT_WAVES * 64) {
    const int cp = task / NPART, part = task % NPART;
    u16x8 o0, o1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const unsigned v = *reinterpret_cast<const unsigned*>(tile + (8 * part + i) * PITCH + 2 * cp);
      o0[i] = (unsigned short)(v & 0xffff);
      o1[i] = (unsigned short)(v >> 16);
    }
    *reinterpret_cast<u16x8*>(yt + (int64_t)(2 * cp) * ldt + r0 + 8 * part) = o0;
    *reinterpret_cast<u16x8*>(yt + (int64_t)(2 * cp + 1) * ldt + r0 + 8 * part) = o1;
  }
}

// A previous backward call's dw partial rows, reduced by this launch (the chained form,
// pico_rmsnorm_bwd_chain): workgroup b sums columns [b * cpw, (b + 1) * cpw) over the `nb` partial rows in a
// fixed order and applies the dw mode, instead of a separate launch of rmsnorm_dw_kernel.
struct DwPrev {
  const float* part;  // nullptr: nothing to reduce
  void* dw;
  int nb, cols, cpw, mode;
  float scale;
};
constexpr int PREV_COLS = 16;  // column slots per workgroup (cpw <= 16)

// Backward: dx = rstd * (g - xhat * mean(g * xhat)), g = dy * w, xhat = x * rstd;
// dw partial per workgroup (deterministic two-stage reduction, no atomics).
// FULL: cols == MAXC * 512 (every lane chunk in range: no per-chunk predicates, which otherwise
// make hipcc spill). NW waves per workgroup (16 up to 1024 columns, 8 up to 2048, 4 above — the
// most that fit without spilling), one row per wave per pass, at most one workgroup per CU; the per-wave dw
// partials accumulate in LDS and the workgroup's sum is one fp32 row per CU. The weight chunks are loaded once
// per wave (loop-invariant). (Measured and removed: two rows per wave per pass, 16.0 -> 16.7 us in the step;
// 16 waves at 2048 columns, 15.3 -> 42.8 us.)
template <int MAXC, int NW, bool FULL, bool RES>
__global__ __launch_bounds__(NW * 64) void rmsnorm_bwd_kernel(const bf16_t* __restrict__ dy,
                                                              const bf16_t* __restrict__ dres,
                                                              const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                              const float* __restrict__ rstd, bf16_t* __restrict__ dx,
                                                              float* __restrict__ dw_part, int64_t rows, int cols,
                                                              const DwPrev prev) {
  __shared__ float red[NW * MAXC * 512];  // per-wave dw partial rows (accumulated in LDS, not registers)
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  // chained dw of the previous call: this thread's partial rows of one column slot, loaded first (in flight
  // during the row loop); slot c = t % 16, row group g = t / 16, rows g, g + NG, ... — and the current value
  // of the target column for the in-place modes (its read is off the kernel's tail too)
  constexpr int NG = NW * 64 / PREV_COLS, PR = 256 / NG;  // prev.nb <= 256 (host check)
  float pv[PR];
  const int pcs = threadIdx.x % PREV_COLS, pg = threadIdx.x / PREV_COLS;
  const int pcol = blockIdx.x * prev.cpw + pcs;
  const bool pok = prev.part && pcs < prev.cpw && pcol < prev.cols;
#pragma unroll
  for (int k = 0; k < PR; ++k) {
    const int pr = pg + NG * k;
    pv[k] = (pok && pr < prev.nb) ? prev.part[(int64_t)pr * prev.cols + pcol] : 0.f;
  }
  float pold = 0.f;
  if (pok && pg == 0 && prev.mode != 0)
    pold = prev.mode == 1 ? bf2f(((const bf16_t*)prev.dw)[pcol]) : ((const float*)prev.dw)[pcol];
  float* myred = red + wid * MAXC * 512 + lane * 8;  // chunk c at + 512 c
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    *reinterpret_cast<f32x4*>(myred + 512 * c) = (f32x4)0.f;
    *reinterpret_cast<f32x4*>(myred + 512 * c + 4) = (f32x4)0.f;
  }
  u16x8 wv[MAXC];  // loop-invariant
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
    if (FULL || (c * 64 + lane) * 8 < cols) wv[c] = *reinterpret_cast<const u16x8*>(w + lane * 8 + 512 * c);
  const int64_t stride = (int64_t)gridDim.x * NW;
#pragma unroll 1
  for (int64_t row = (int64_t)blockIdx.x * NW + wid; row < rows; row += stride) {
    u16x8 xv[MAXC], dv[MAXC], rv[MAXC];
    const float rs = rstd[row];
    const int64_t ro = row * cols + lane * 8;  // this lane's first element of the row; chunk c at + 512 c
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (FULL || (c * 64 + lane) * 8 < cols) {
        xv[c] = *reinterpret_cast<const u16x8*>(x + ro + 512 * c);
        dv[c] = *reinterpret_cast<const u16x8*>(dy + ro + 512 * c);
        if constexpr (RES) rv[c] = *reinterpret_cast<const u16x8*>(dres + ro + 512 * c);
      }
    }
    float dot = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (FULL || (c * 64 + lane) * 8 < cols) {
        f32x4 a = *reinterpret_cast<const f32x4*>(myred + 512 * c);
        f32x4 bq = *reinterpret_cast<const f32x4*>(myred + 512 * c + 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = bf2f(xv[c][j]) * rs, d = bf2f(dv[c][j]);
          if (j < 4) a[j] += d * xh;
          else bq[j - 4] += d * xh;
          dot += d * bf2f(wv[c][j]) * xh;
        }
        *reinterpret_cast<f32x4*>(myred + 512 * c) = a;
        *reinterpret_cast<f32x4*>(myred + 512 * c + 4) = bq;
      }
    }
    dot = wave_sum(dot) / (float)cols;
    bf16_t* dxr = dx + ro;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (FULL || (c * 64 + lane) * 8 < cols) {
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = bf2f(xv[c][j]) * rs;
          float v = rs * (bf2f(dv[c][j]) * bf2f(wv[c][j]) - xh * dot);
          if constexpr (RES) v += bf2f(rv[c][j]);
          o[j] = f2bf(v);
        }
        *reinterpret_cast<u16x8*>(dxr + 512 * c) = o;
      }
    }
  }
  // reduce the NW waves' dw partials (fixed order), one fp32 row per workgroup
  __syncthreads();
  for (int col = threadIdx.x; col < cols; col += NW * 64) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) s += red[k * MAXC * 512 + col];
    dw_part[(int64_t)blockIdx.x * cols + col] = s;
  }
  if (prev.part) {  // workgroup-uniform: the previous call's dw, columns of this workgroup's slice
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < PR; ++k) s += pv[k];  // rows ascending
    // the wave's four row groups of one column slot (lanes pcs, +16, +32, +48): ((g0 + g1) + (g2 + g3))
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    __syncthreads();  // every thread past its reads of red
    if (lane < PREV_COLS) red[wid * PREV_COLS + lane] = s;
    __syncthreads();
    if (threadIdx.x < prev.cpw && blockIdx.x * prev.cpw + (int)threadIdx.x < prev.cols) {
      const int col = blockIdx.x * prev.cpw + threadIdx.x;
      float t = 0.f;
#pragma unroll
      for (int g = 0; g < NW; ++g) t += red[g * PREV_COLS + threadIdx.x];  // waves ascending: fixed order
      if (prev.mode == 0) {
        ((bf16_t*)prev.dw)[col] = f2bf(t);
      } else if (prev.mode == 1) {
        ((bf16_t*)prev.dw)[col] = f2bf(pold + t);
      } else {
        ((float*)prev.dw)[col] = (pold + t) * prev.scale;
      }
    }
  }
}

constexpr int bwd_waves(int maxc) { return maxc <= 2 ? 16 : (maxc == 4 ? 8 : 4); }

template <int M>
int launch_rmsnorm_bwd(const void* dy, const void* dres, const void* x, const void* w, const float* rstd, void* dx,
                       float* part, int64_t rows, int c, int nb, const DwPrev& prev, hipStream_t s) {
  constexpr int NW = bwd_waves(M);
  auto go = [&](auto full, auto res) {
    PICO_TRY(pico_launch(PICO_K_RMSNORM_BWD, "rmsnorm_bwd", rmsnorm_bwd_kernel<M, NW, decltype(full)::value, decltype(res)::value>, dim3(nb), dim3(NW * 64), 0, s, (const bf16_t*)dy, (const bf16_t*)dres, (const bf16_t*)x, (const bf16_t*)w, rstd, (bf16_t*)dx,
                    part, rows, c, prev));
    return 0;
  };
  const bool full = c == M * 512;
  if (full && dres) return go(std::true_type{}, std::true_type{});
  if (full) return go(std::true_type{}, std::false_type{});
  if (dres) return go(std::false_type{}, std::true_type{});
  return go(std::false_type{}, std::false_type{});
}

// dw[col] = sum over the workgroup partials, in a fixed order (deterministic): a 256-thread
// workgroup covers DW_COLS columns x (256 / DW_COLS) row-slices; each thread sums its slice (loads
// coalesced across the columns), then the slices are combined through LDS in slice order.
// MODE 0: dw (bf16) = sum; 1: dw (bf16) = bf16(dw + sum); 2: dw (fp32) = (dw + sum) * scale
#ifndef PICO_RMS_DW_COLS
#define PICO_RMS_DW_COLS 32
#endif
constexpr int DW_COLS = PICO_RMS_DW_COLS, DW_SL = 256 / DW_COLS;

template <int MODE>
__global__ __launch_bounds__(256) void rmsnorm_dw_kernel(const float* __restrict__ part, void* __restrict__ dw, int nblk,
                                                         int cols, float scale) {
  __shared__ float red[DW_SL][DW_COLS];
  const int c = threadIdx.x % DW_COLS, sl = threadIdx.x / DW_COLS;
  const int col = blockIdx.x * DW_COLS + c;
  float s = 0.f;
  if (col < cols) {
#pragma unroll 8
    for (int b = sl; b < nblk; b += DW_SL) s += part[(int64_t)b * cols + col];
  }
  red[sl][c] = s;
  __syncthreads();
  if (sl == 0 && col < cols) {
    float t = red[0][c];
#pragma unroll
    for (int k = 1; k < DW_SL; ++k) t += red[k][c];
    if constexpr (MODE == 0) {
      ((bf16_t*)dw)[col] = f2bf(t);
    } else if constexpr (MODE == 1) {
      bf16_t* p = (bf16_t*)dw + col;
      *p = f2bf(bf2f(*p) + t);
    } else {
      float* p = (float*)dw + col;
      *p = (*p + t) * scale;
    }
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


#ifndef PICO_RMS_BWD_MAXB
#define PICO_RMS_BWD_MAXB 256
#endif

int bwd_blocks(int64_t rows, int64_t cols) {  // one workgroup per CU at most: few dw partial rows
  const int nw = bwd_waves(maxc_for(cols));
  int64_t nb = (rows + nw - 1) / nw;
  return (int)(nb < PICO_RMS_BWD_MAXB ? nb : PICO_RMS_BWD_MAXB);
}

}  // namespace

extern "C" {

int pico_rmsnorm_fwd_t(const void* x, const void* residual, const void* weight, void* y, void* residual_out,
                       float* rstd, void* y_t, int64_t ld_t, int64_t rows, int64_t cols, float eps, void* stream) {
  PICO_REQUIRE(x && weight && y && rstd && y_t, "pico_rmsnorm_fwd_t: null pointer");
  PICO_REQUIRE(cols == 1024 || cols == 2048, "pico_rmsnorm_fwd_t: cols=%lld unsupported (1024 or 2048)",
               (long long)cols);
  PICO_REQUIRE(rows >= 0 && rows % 32 == 0 && ld_t >= rows && ld_t % 8 == 0,
               "pico_rmsnorm_fwd_t: rows must be a multiple of 32 and ld_t >= rows, multiple of 8");
  PICO_REQUIRE((((uintptr_t)x | (uintptr_t)y | (uintptr_t)y_t | (uintptr_t)weight | (uintptr_t)residual |
                 (uintptr_t)residual_out) & 15) == 0,
               "pico_rmsnorm_fwd_t: pointers must be 16-byte aligned");
  PICO_REQUIRE(rows / 32 < (1ll << 31), "pico_rmsnorm_fwd_t: too many rows");
  if (rows == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)(rows / FWDT_ROWS);
  const size_t lds = FWDT_ROWS * (cols + 8) * 2;
  auto xp = (const bf16_t*)x;
  auto rp = (const bf16_t*)residual;
  auto wp = (const bf16_t*)weight;
  auto go = [&](auto maxc, auto res) {
    constexpr int M = decltype(maxc)::value;
    constexpr bool R = decltype(res)::value;
    auto k = rmsnorm_fwd_t_kernel<M, R>;
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return pico_set_error("pico_rmsnorm_fwd_t: cannot set LDS size (%d)", (int)e);
    PICO_TRY(pico_launch(PICO_K_RMSNORM_FWD, "rmsnorm_fwd_t", k, dim3(nb), dim3(FWDT_WAVES * 64), lds, s, xp, rp, wp, (bf16_t*)y, (bf16_t*)residual_out, rstd, (bf16_t*)y_t, ld_t, eps));
    return 0;
  };
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;
  if (cols == 2048) return residual ? go(I4{}, std::true_type{}) : go(I4{}, std::false_type{});
  return residual ? go(I2{}, std::true_type{}) : go(I2{}, std::false_type{});
}

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
    PICO_TRY(pico_launch(PICO_K_RMSNORM_FWD, "rmsnorm_fwd", rmsnorm_fwd_kernel<M>, dim3(grid), dim3(block), 0, s, xp, rp, wp, yp, rop, rstd, rows, c, eps)); \
    break;
  switch (mc) {
    FWD_CASE(1) FWD_CASE(2) FWD_CASE(4) FWD_CASE(8) FWD_CASE(16)
  }
#undef FWD_CASE
  return 0;
}

int64_t pico_rmsnorm_bwd_workspace_bytes(int64_t rows, int64_t cols) {
  if (maxc_for(cols) <= 0) return 0;
  return (int64_t)bwd_blocks(rows, cols) * cols * (int64_t)sizeof(float);
}

int pico_rmsnorm_bwd(const void* dy, const void* dresidual, const void* x, const void* weight, const float* rstd,
                     void* dx, void* dweight, void* workspace, int64_t rows, int64_t cols, void* stream) {
  return pico_rmsnorm_bwd_acc(dy, dresidual, x, weight, rstd, dx, dweight, 0, 1.f, workspace, rows, cols, stream);
}

int pico_rmsnorm_bwd_acc(const void* dy, const void* dresidual, const void* x, const void* weight, const float* rstd,
                         void* dx, void* dweight, int dw_mode, float dw_scale, void* workspace, int64_t rows,
                         int64_t cols, void* stream) {
  return pico_rmsnorm_bwd_chain(dy, dresidual, x, weight, rstd, dx, dweight, dw_mode, dw_scale, workspace, rows, cols,
                                1, nullptr, 0, 0, nullptr, 0, 1.f, stream);
}

int pico_rmsnorm_dw_reduce(const float* part, int64_t nb, int64_t cols, void* dweight, int dw_mode, float dw_scale,
                           void* stream) {
  PICO_REQUIRE(part && dweight, "pico_rmsnorm_dw_reduce: null pointer");
  PICO_REQUIRE(dw_mode >= 0 && dw_mode <= 2, "pico_rmsnorm_dw_reduce: dw_mode %d not in 0..2", dw_mode);
  PICO_REQUIRE(nb > 0 && cols > 0 && nb < (1 << 30) && cols < (1 << 30), "pico_rmsnorm_dw_reduce: bad shape");
  hipStream_t s = (hipStream_t)stream;
  const int g = pico_cdiv(cols, DW_COLS), n = (int)nb, c = (int)cols;
  if (dw_mode == 0) {
    PICO_TRY(pico_launch(PICO_K_RMSNORM_DW, "rmsnorm_dw", rmsnorm_dw_kernel<0>, dim3(g), dim3(256), 0, s, part, dweight, n, c, 1.f));
  } else if (dw_mode == 1) {
    PICO_TRY(pico_launch(PICO_K_RMSNORM_DW, "rmsnorm_dw", rmsnorm_dw_kernel<1>, dim3(g), dim3(256), 0, s, part, dweight, n, c, 1.f));
  } else {
    PICO_TRY(pico_launch(PICO_K_RMSNORM_DW, "rmsnorm_dw", rmsnorm_dw_kernel<2>, dim3(g), dim3(256), 0, s, part, dweight, n, c, dw_scale));
  }
  return 0;
}

int64_t pico_rmsnorm_bwd_partial_rows(int64_t rows, int64_t cols) {
  return maxc_for(cols) > 0 ? bwd_blocks(rows, cols) : 0;
}

int pico_rmsnorm_bwd_chain(const void* dy, const void* dresidual, const void* x, const void* weight, const float* rstd,
                           void* dx, void* dweight, int dw_mode, float dw_scale, void* workspace, int64_t rows,
                           int64_t cols, int reduce_own, const float* prev_part, int64_t prev_nb, int64_t prev_cols,
                           void* prev_dweight, int prev_mode, float prev_scale, void* stream) {
  PICO_REQUIRE(dy && x && weight && rstd && dx && workspace && (dweight || !reduce_own), "pico_rmsnorm_bwd: null pointer");
  PICO_REQUIRE(dw_mode >= 0 && dw_mode <= 2, "pico_rmsnorm_bwd_acc: dw_mode %d not in 0..2", dw_mode);
  PICO_REQUIRE(rows > 0 && cols > 0 && cols % 8 == 0, "pico_rmsnorm_bwd: bad shape rows=%lld cols=%lld",
               (long long)rows, (long long)cols);
  const int mc = maxc_for(cols);
  PICO_REQUIRE(mc > 0 && mc <= 8, "pico_rmsnorm_bwd: cols=%lld > 4096 unsupported", (long long)cols);
  hipStream_t s = (hipStream_t)stream;
  const int nb = bwd_blocks(rows, cols);
  DwPrev prev{nullptr, nullptr, 0, 0, 0, 0, 1.f};
  if (prev_part) {
    PICO_REQUIRE(prev_dweight && prev_mode >= 0 && prev_mode <= 2 && prev_nb > 0 && prev_nb <= 256 && prev_cols > 0,
                 "pico_rmsnorm_bwd_chain: bad previous partials");
    const int64_t cpw = (prev_cols + nb - 1) / nb;
    if (cpw <= PREV_COLS) {
      prev = DwPrev{prev_part, prev_dweight, (int)prev_nb, (int)prev_cols, (int)cpw, prev_mode, prev_scale};
    } else {  // too many columns for this grid: reduce them in their own launch first
      PICO_TRY(pico_rmsnorm_dw_reduce(prev_part, prev_nb, prev_cols, prev_dweight, prev_mode, prev_scale, stream));
    }
  }
  auto part = (float*)workspace;
  const int c = (int)cols;
  int rc = 0;
  switch (mc) {
    case 1: rc = launch_rmsnorm_bwd<1>(dy, dresidual, x, weight, rstd, dx, part, rows, c, nb, prev, s); break;
    case 2: rc = launch_rmsnorm_bwd<2>(dy, dresidual, x, weight, rstd, dx, part, rows, c, nb, prev, s); break;
    case 4: rc = launch_rmsnorm_bwd<4>(dy, dresidual, x, weight, rstd, dx, part, rows, c, nb, prev, s); break;
    case 8: rc = launch_rmsnorm_bwd<8>(dy, dresidual, x, weight, rstd, dx, part, rows, c, nb, prev, s); break;
  }
  if (rc) return rc;
  if (reduce_own) return pico_rmsnorm_dw_reduce(part, nb, cols, dweight, dw_mode, dw_scale, stream);
  return 0;
}

}  // extern "C"
