// Rotary position embedding (rotate-half / non-interleaved layout), forward and backward.
//
// Replaces flash-attn's Triton apply_rotary_emb(x, cos[:, :D/2], sin[:, :D/2], interleaved=False)
// called from Attention.forward (ref picotron/model.py:135-136); the eager oracle is
// apply_rotary_pos_emb (ref picotron/model.py:12-19) with tables from get_cos_sin (:21-30).
// fp32 math on the bf16 inputs and bf16 tables, one rounding per output element. The backward
// is the same rotation by -theta (conjugate = 1).
//
// Each thread owns 8 consecutive rotary pairs: two 16-byte loads of x (i and i + D/2), two of the
// tables, two 16-byte stores. Algorithmic bytes: 2 * 2 B per element of x (tables are L2-resident).
#include "common.h"

namespace {

// n / d for 0 <= n < 2^31 by a multiply-high (round-up method; m and l precomputed on the host): the rope
// thread's index decomposition otherwise costs three 32-bit integer divisions (~40 VALU each), a sizeable
// share of a kernel that issues four 16-byte loads per thread
struct FastDiv {
  unsigned d, m, l;
};
FastDiv make_fastdiv(unsigned d) {
  FastDiv f;
  f.d = d;
  f.l = 0;
  while ((1ull << f.l) < d) ++f.l;
  f.m = (unsigned)((((1ull << 32) * ((1ull << f.l) - d)) / d) + 1);
  return f;
}
PICO_DEV unsigned fdiv(unsigned n, const FastDiv& f) { return (__umulhi(n, f.m) + n) >> f.l; }

// t enumerates (b, s, head, vector) with the vector fastest, so a wave's loads and stores cover whole rows.
// (Measured and removed: two heads per thread sharing the cos / sin loads, 5.7 vs 5.6 us; streaming loads,
// 9.6 vs 9.1 us in the step.)
__global__ __launch_bounds__(256) void rope_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ out,
                                                   const bf16_t* __restrict__ cosp, const bf16_t* __restrict__ sinp,
                                                   int64_t total, FastDiv fv, FastDiv fh, FastDiv fs, int half,
                                                   int64_t xs0, int64_t xs1, int64_t xs2, int64_t os0, int64_t os1,
                                                   int64_t os2, int64_t cs, float sign) {
  for (unsigned t = blockIdx.x * 256 + threadIdx.x; t < (unsigned)total; t += gridDim.x * 256) {
    const unsigned r0 = fdiv(t, fv);  // (b, s, head) row; vector vi of 8 pairs within it
    const int vi = (int)(t - r0 * fv.d);
    const unsigned r1 = fdiv(r0, fh);  // fh.d = heads
    const int hd = (int)(r0 - r1 * fh.d);
    const unsigned b = fdiv(r1, fs);
    const int s = (int)(r1 - b * fs.d);
    const int i = vi * 8;
    const u16x8 c = *reinterpret_cast<const u16x8*>(cosp + (int64_t)s * cs + i);
    const u16x8 sn = *reinterpret_cast<const u16x8*>(sinp + (int64_t)s * cs + i);
    const bf16_t* xp = x + (int64_t)b * xs0 + (int64_t)s * xs1 + (int64_t)hd * xs2 + i;
    const u16x8 x1 = *reinterpret_cast<const u16x8*>(xp);
    const u16x8 x2 = *reinterpret_cast<const u16x8*>(xp + half);
    {
      u16x8 o1, o2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = bf2f(x1[j]), bb = bf2f(x2[j]);
        const float cf = bf2f(c[j]), sf = sign * bf2f(sn[j]);
        // products rounded before the sum (no FMA contraction: flash-attn's fp32 rotary / the oracle's
        // restatement, and the same arithmetic as the q rotation inside the attention forward)
        o1[j] = f2bf(__fmul_rn(a, cf) - __fmul_rn(bb, sf));
        o2[j] = f2bf(__fmul_rn(bb, cf) + __fmul_rn(a, sf));
      }
      bf16_t* op = out + (int64_t)b * os0 + (int64_t)s * os1 + (int64_t)hd * os2 + i;
      *reinterpret_cast<u16x8*>(op) = o1;
      *reinterpret_cast<u16x8*>(op + half) = o2;
    }
  }
}

}  // namespace

extern "C" int pico_rope(const void* x, void* out, const void* cos, const void* sin, int64_t batch, int64_t seqlen,
                         int64_t heads, int64_t head_dim, const int64_t* xst, const int64_t* ost, int64_t cs_stride,
                         int conjugate, void* stream) {
  PICO_REQUIRE(x && out && cos && sin && xst && ost, "pico_rope: null pointer");
  PICO_REQUIRE(head_dim % 16 == 0 && head_dim > 0, "pico_rope: head_dim=%lld must be a multiple of 16",
               (long long)head_dim);
  PICO_REQUIRE(((uintptr_t)x | (uintptr_t)out | (uintptr_t)cos | (uintptr_t)sin) % 16 == 0,
               "pico_rope: pointers must be 16-byte aligned");
  for (int d = 0; d < 3; ++d)
    PICO_REQUIRE(xst[d] % 8 == 0 && ost[d] % 8 == 0, "pico_rope: strides must be multiples of 8 elements");
  PICO_REQUIRE(cs_stride % 8 == 0 && cs_stride >= head_dim / 2, "pico_rope: bad cos/sin row stride %lld",
               (long long)cs_stride);
  const int64_t total = batch * seqlen * heads * (head_dim / 16);
  PICO_REQUIRE(total < (int64_t)0x7fffffff, "pico_rope: tensor too large");
  if (total == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  int64_t nb = (total + 255) / 256;
  if (nb > 8192) nb = 8192;
  PICO_TRY(pico_launch(PICO_K_ROPE, "rope", rope_kernel, dim3((int)nb), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)out,
                       (const bf16_t*)cos, (const bf16_t*)sin, total, make_fastdiv((unsigned)(head_dim / 16)),
                       make_fastdiv((unsigned)heads), make_fastdiv((unsigned)seqlen), (int)(head_dim / 2), xst[0],
                       xst[1], xst[2], ost[0], ost[1], ost[2], cs_stride, conjugate ? -1.f : 1.f));
  return 0;
}
