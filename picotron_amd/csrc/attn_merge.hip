// Ring-attention block merge (update_out_and_lse, ref picotron/context_parallel/context_parallel.py:157-187):
//   first block:  out = float(block_out), lse = block_lse
//   otherwise:    out = out - sigmoid(block_lse - lse) * (out - block_out)
//                 lse = lse - logsigmoid(lse - block_lse)
// Every operand is addressed by element strides, so one kernel serves the reference's layout (out
// [B, H, S, D] fp32, lse [B, H, S, 1], possibly sliced views, ref :183-186) and the ring's internal one
// (out [B, S, H, D]): out fp32 (strides b, s, h; unit d), lse fp32 (strides b, h, s), block_out bf16 or fp32
// (strides b, s, h; unit d), block_lse fp32 (strides b, h, s). D/8 lanes per (b, s, h) row, 8 elements each
// (HBM-bound: 4+4+2 B per element, plus 12 B per row).
#include "common.h"

namespace {

struct MergeStrides {
  int64_t o[3], l[3], bo[3], bl[3];
};

template <bool BO_F32>
__global__ __launch_bounds__(256) void attn_merge_kernel(float* __restrict__ out, float* __restrict__ lse,
                                                         const void* __restrict__ bo_, const float* __restrict__ blse,
                                                         int B, int S, int H, int D, MergeStrides st, int first) {
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
  float bv[8];
  if constexpr (BO_F32) {
    const float* p = (const float*)bo_ + b * st.bo[0] + s * st.bo[1] + h * st.bo[2] + sub * 8;
    const f32x4 x0 = reinterpret_cast<const f32x4*>(p)[0], x1 = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bv[j] = x0[j];
      bv[4 + j] = x1[j];
    }
  } else {
    const u16x8 x = *reinterpret_cast<const u16x8*>((const bf16_t*)bo_ + b * st.bo[0] + s * st.bo[1] + h * st.bo[2] +
                                                    sub * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) bv[j] = bf2f(x[j]);
  }
  f32x4* op = reinterpret_cast<f32x4*>(out + b * st.o[0] + s * st.o[1] + h * st.o[2] + sub * 8);
  float* lp = lse + b * st.l[0] + h * st.l[1] + s * st.l[2];
  const float bl = blse[b * st.bl[0] + h * st.bl[1] + s * st.bl[2]];
  if (first) {
    op[0] = f32x4{bv[0], bv[1], bv[2], bv[3]};
    op[1] = f32x4{bv[4], bv[5], bv[6], bv[7]};
    if (sub == 0) *lp = bl;
    return;
  }
  const float l = *lp;
  const float wgt = 1.f / (1.f + expf(-(bl - l)));  // sigmoid(block_lse - lse)
  f32x4 a = op[0], c = op[1];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    a[j] = a[j] - wgt * (a[j] - bv[j]);
    c[j] = c[j] - wgt * (c[j] - bv[4 + j]);
  }
  op[0] = a;
  op[1] = c;
  if (sub == 0) {
    const float x = l - bl;  // logsigmoid(x) = min(x, 0) - log1p(exp(-|x|))
    const float ls = fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
    *lp = l - ls;
  }
}

}  // namespace

extern "C" int pico_attn_merge(float* out, const int64_t* out_strides, float* lse, const int64_t* lse_strides,
                               const void* block_out, const int64_t* block_out_strides, int block_out_f32,
                               const float* block_lse, const int64_t* block_lse_strides, int64_t batch, int64_t seqlen,
                               int64_t heads, int64_t head_dim, int first, void* stream) {
  PICO_REQUIRE(out && lse && block_out && block_lse, "pico_attn_merge: null pointer");
  PICO_REQUIRE(out_strides && lse_strides && block_out_strides && block_lse_strides, "pico_attn_merge: null strides");
  PICO_REQUIRE(head_dim % 8 == 0 && head_dim <= 256, "pico_attn_merge: bad head_dim");
  for (int d = 0; d < 3; ++d) {
    PICO_REQUIRE(block_out_strides[d] % (block_out_f32 ? 4 : 8) == 0 && out_strides[d] % 4 == 0,
                 "pico_attn_merge: out / block_out strides must keep 16-byte alignment");
  }
  PICO_REQUIRE(((uintptr_t)out | (uintptr_t)block_out) % 16 == 0, "pico_attn_merge: out / block_out must be 16-byte aligned");
  const int64_t threads = batch * seqlen * heads * (head_dim / 8);
  if (threads == 0) return 0;
  MergeStrides st;
  for (int d = 0; d < 3; ++d) {
    st.o[d] = out_strides[d];
    st.l[d] = lse_strides[d];
    st.bo[d] = block_out_strides[d];
    st.bl[d] = block_lse_strides[d];
  }
  hipStream_t s = (hipStream_t)stream;
  if (block_out_f32) {
    PICO_TRY(pico_launch(PICO_K_ATTN_MERGE, "attn_merge", attn_merge_kernel<true>, dim3(pico_cdiv(threads, 256)), dim3(256), 0,
                         s, out, lse, block_out, block_lse, (int)batch, (int)seqlen, (int)heads, (int)head_dim, st, first));
  } else {
    PICO_TRY(pico_launch(PICO_K_ATTN_MERGE, "attn_merge", attn_merge_kernel<false>, dim3(pico_cdiv(threads, 256)), dim3(256), 0,
                         s, out, lse, block_out, block_lse, (int)batch, (int)seqlen, (int)heads, (int)head_dim, st, first));
  }
  return 0;
}
