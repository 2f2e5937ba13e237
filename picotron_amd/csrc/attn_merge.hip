// Ring-attention block merge (update_out_and_lse, ref picotron/context_parallel/context_parallel.py:157-187):
//   first block:  out = float(block_out), lse = block_lse
//   otherwise:    out = out - sigmoid(block_lse - lse) * (out - block_out)
//                 lse = lse - logsigmoid(lse - block_lse)
// out fp32 [B, S, H, D] contiguous, lse fp32 [B, H, S], block_out bf16 [B, S, H, D] (strided rows),
// block_lse fp32 [B, H, S]. D/8 lanes per (b, s, h) row, 8 elements each (HBM-bound:
// 4+4+2 B per element, plus 12 B per row).
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void attn_merge_kernel(float* __restrict__ out, float* __restrict__ lse,
                                                         const bf16_t* __restrict__ bo, const float* __restrict__ blse,
                                                         int B, int S, int H, int D, int64_t bs0, int64_t bs1,
                                                         int64_t bs2, int first) {
  const int lpr = D / 8;
  const int64_t rows = (int64_t)B * S * H;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = gid / lpr;
  const int sub = (int)(gid % lpr);
  if (row >= rows) return;
  const int h = (int)(row % H);
  const int64_t bsr = row / H;
  const int s = (int)(bsr % S);
  const int b = (int)(bsr / S);
  const int64_t li = ((int64_t)b * H + h) * S + s;
  const u16x8 bv = *reinterpret_cast<const u16x8*>(bo + b * bs0 + s * bs1 + h * bs2 + sub * 8);
  f32x4* op = reinterpret_cast<f32x4*>(out + row * D + sub * 8);
  const float bl = blse[li];
  if (first) {
    f32x4 a, c;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] = bf2f(bv[j]);
      c[j] = bf2f(bv[4 + j]);
    }
    op[0] = a;
    op[1] = c;
    if (sub == 0) lse[li] = bl;
    return;
  }
  const float l = lse[li];
  const float wgt = 1.f / (1.f + expf(-(bl - l)));  // sigmoid(block_lse - lse)
  f32x4 a = op[0], c = op[1];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    a[j] = a[j] - wgt * (a[j] - bf2f(bv[j]));
    c[j] = c[j] - wgt * (c[j] - bf2f(bv[4 + j]));
  }
  op[0] = a;
  op[1] = c;
  if (sub == 0) {
    const float x = l - bl;  // logsigmoid(x) = min(x, 0) - log1p(exp(-|x|))
    const float ls = fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
    lse[li] = l - ls;
  }
}

}  // namespace

extern "C" int pico_attn_merge(float* out, float* lse, const void* block_out, const float* block_lse, int64_t batch,
                               int64_t seqlen, int64_t heads, int64_t head_dim, const int64_t* bo_strides, int first,
                               void* stream) {
  PICO_REQUIRE(out && lse && block_out && block_lse && bo_strides, "pico_attn_merge: null pointer");
  PICO_REQUIRE(head_dim % 8 == 0 && head_dim <= 256, "pico_attn_merge: bad head_dim");
  for (int d = 0; d < 3; ++d) PICO_REQUIRE(bo_strides[d] % 8 == 0, "pico_attn_merge: strides must be multiples of 8");
  const int64_t threads = batch * seqlen * heads * (head_dim / 8);
  if (threads == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  PICO_TRY(pico_launch(PICO_K_ATTN_MERGE, "attn_merge", attn_merge_kernel, dim3(pico_cdiv(threads, 256)), dim3(256), 0, s, out, lse, (const bf16_t*)block_out, block_lse, (int)batch, (int)seqlen, (int)heads, (int)head_dim,
                  bo_strides[0], bo_strides[1], bo_strides[2], first));
  return 0;
}
