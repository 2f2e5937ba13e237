// Flash-attention backward, dQ kernel for head_dim 64 on gfx950: the tile-pipelined form.
//
// Same contract as attn_bwd_q_kernel<64> (attn_bwd_split.hip), which it replaces when PICO_ATTN_BWDQ64 = 1:
// one workgroup = 4 waves = 128 query rows of one (batch, q-head), sweeping 64-key tiles of K | V (LDS-DMA
// ring, the same swizzled images and piece map); S^T = K Q^T and dP^T = V dO^T with the query on the lane,
// P^T = exp2(S scale log2e - LSE log2e), dS^T = P^T (dP^T - delta), dQ^T += K^T dS^T (transposed reads of
// the K image); it also writes LSE log2e and -delta for the dK/dV kernel, and applies RoPE^-1 / the fp32
// accumulate mode in its epilogue. Replaces part of flash-attn's backward of flash_attn_func (ref
// picotron/model.py:32-36) and of the ring block backward (ref picotron/context_parallel/context_parallel.py:130-155).
//
// Why: the 24 MFMAs of a tile (768 matrix cycles) against ~140 VALU (~560 issue cycles) make the kernel
// MFMA-bound in principle, but attn_bwd_q_kernel runs each tile as S / dP MFMAs -> dependent softmax VALU ->
// dQ MFMAs, and measured 26 % MFMA busy (PMC) at three workgroups per CU. Here each wave pipelines across
// tiles: interval t issues the S / dP MFMAs of tile t + 1 and the dQ MFMAs of tile t, with the VALU of tile
// t (P, dS, bf16 packing) between them, in a hand-ordered 24-slot schedule (sched_barrier(0) fences; every
// operand read three slots ahead). S / dP of two tiles alternate between two named register sets (the loop
// is unrolled by two). 256 VGPRs, 64 KiB LDS: two workgroups per CU.
#include "attn_common.h"

// PICO_BQ64_ABL: ablation builds for timing only (results wrong): 1 no operand LDS reads, 2 no softmax VALU,
// 4 no tile wait / barrier, 8 no M1 MFMAs, 16 no dQ MFMAs, 32 no DMA in the loop (stale tiles), 64 the softmax VALU
// without dependencies (same op counts, every op reads S / dP), 128 exp2 replaced by a plain multiply
#ifndef PICO_BQ64_ABL
#define PICO_BQ64_ABL 0
#endif
#ifndef PICO_BQ64_RD
#define PICO_BQ64_RD 3  // operand reads issued this many MFMA slots ahead of their consumer
#endif

namespace {

constexpr int QB = 128, KT = 64, D = 64, KS = 4, DT = 2, RB = 2 * D;
constexpr int IMG = KT * RB;       // one K (or V) tile image, lds_off<64> layout
constexpr int SLOT = 2 * IMG;      // K | V
constexpr int NBUF = 4;            // ring slots; prefetch distance 2 tiles
constexpr int NP = SLOT / 1024;    // 1-KiB DMA pieces per tile (16)
constexpr int NPW = NP / 4;        // per wave
constexpr int RPP = 1024 / RB;     // image rows per piece
constexpr int CPR = D / 8;         // 16-byte chunks per row

// The 24 MFMA slots of an interval: values < 16 are the M1 MFMAs of tile t + 1 (0-7: S^T, kt = i / 4,
// ks = i % 4; 8-15: dP^T), 16 + 2 c + dt the dQ MFMA of chunk c = (kt, st) of tile t, placed right after the
// slot in which the chunk's last cvt_pk issues (7 VALU ops per slot: chunk c ends in slot 5 + 5c - (c > 0)).
constexpr int bq_slot(int s) {
  const int t[24] = {0, 1, 2, 3, 4, 5, 16, 17, 6, 7, 8, 18, 19, 9, 10, 11, 20, 21, 12, 13, 14, 22, 23, 15};
  return t[s];
}
// VALU op j (0..35) of a chunk of 8 keys: 100 * type + index, type 0 f (t = fma(S, scale log2e, -LSE log2e)),
// 1 e (p = exp2(t)), 2 a (d = dP - delta), 3 m (ds = p d), 4 v (cvt_pk pair of ds); every consumer at least
// two ops after its producers.
constexpr int bq_op(int j) {
  const int seq[36] = {0,   1,   2,   3,   100, 101, 102, 103, 4,   5,   6,   7,   200, 201, 202, 203, 300, 301,
                       302, 303, 104, 105, 106, 107, 204, 205, 206, 207, 400, 401, 304, 305, 306, 307, 402, 403};
  return seq[j];
}
constexpr int NVALU = 4 * 36;
constexpr int bq_first_op(int s) { return 7 * s < NVALU ? 7 * s : NVALU; }
constexpr int bq_end_op(int s) { return 7 * (s + 1) < NVALU ? 7 * (s + 1) : NVALU; }
static_assert(bq_slot(6) == 16 && (36 * 1 - 1) / 7 < 6 && (36 * 2 - 1) / 7 < 11 && (36 * 3 - 1) / 7 < 16 &&
                  (36 * 4 - 1) / 7 < 21,
              "each chunk's dQ MFMAs follow its last VALU slot");

PICO_DEV bf16x8 tr_pair_q64(const char* base, unsigned lo_off, unsigned hi_off) {
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + lo_off));
  const i16x4 up = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + hi_off));
  typedef __attribute__((ext_vector_type(8))) short i16x8;
  i16x8 v = {lo[0], lo[1], lo[2], lo[3], up[0], up[1], up[2], up[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <bool CAUSAL>
__global__ __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2)))
void attn_bwd_q64_kernel(const pico_attn_args a, float scale, float scale_log2, float* __restrict__ lse2_g,
                         float* __restrict__ delta_g, int sq_pad, int nfront) {
  __shared__ __attribute__((aligned(16))) char smem[NBUF * SLOT];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int Sq = (int)a.seqlen_q, Sk = (int)a.seqlen_k;

  // causal dispatch order as attn_bwd_q_kernel: the `nfront` lightest query blocks first, then heaviest-first
  const int nmb = (Sq + QB - 1) / QB;
  const int nbh = (int)(a.batch * a.heads_q);
  const int lin = blockIdx.x;
  const int gi = lin / nbh;
  const int mb = !CAUSAL ? gi : (gi < nfront ? gi : nmb - 1 - (gi - nfront));
  const int bh = lin % nbh;
  const int b = bh / (int)a.heads_q, hq = bh % (int)a.heads_q;
  const int hk = hq / (int)(a.heads_q / a.heads_kv);
  const int q0 = mb * QB, qw = q0 + 32 * wave, my_q = qw + r;
  const int qc = min(my_q, Sq - 1);

  const bf16_t* kg = (const bf16_t*)a.k + b * a.k_strides[0] + hk * a.k_strides[2];
  const bf16_t* vg = (const bf16_t*)a.v + b * a.v_strides[0] + hk * a.v_strides[2];
  const int ksd = (int)a.k_strides[1], vsd = (int)a.v_strides[1];

  const int kend = CAUSAL ? min(Sk, q0 + QB) : Sk;
  const int ntiles = (kend + KT - 1) / KT;  // the workgroup's tiles
  const int lim_last = CAUSAL ? min(qw + 31, Sk - 1) : Sk - 1;
  const int lim_first = CAUSAL ? min(qw, Sk - 1) : Sk - 1;
  const int lim_lane = CAUSAL ? min(my_q, Sk - 1) : Sk - 1;
  const int tl = lim_last / KT;  // the wave's last tile (rows qw .. qw + 31 lie in one 64-key tile)

  // ---- DMA (attn_bwd_q_kernel's map): piece j = wave + 4 i; j < 8: K image piece j, else V piece j - 8 ----
  auto piece_row = [&](int i) __attribute__((always_inline)) { return RPP * ((wave + 4 * i) & 7) + lane / CPR; };
  unsigned full_off[NPW];
#pragma unroll
  for (int i = 0; i < NPW; ++i) {
    const int row = piece_row(i);
    full_off[i] = 2u * (unsigned)(row * (i < 2 ? ksd : vsd) + 8 * ((lane % CPR) ^ swz<D>(row)));
  }
  const unsigned smem_lds = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr(smem));
  auto issue = [&](int tile) __attribute__((always_inline)) {
    const unsigned slot = smem_lds + (unsigned)(tile & (NBUF - 1)) * (unsigned)SLOT;
    const int base = tile * KT;
    const bf16_t* kt_ = kg + (int64_t)base * ksd;
    const bf16_t* vt_ = vg + (int64_t)base * vsd;
    const bool full = base + KT <= Sk;
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int jj = (wave + 4 * i) & 7;
      const unsigned dst = slot + (i < 2 ? 0u : (unsigned)IMG) + (unsigned)jj * 1024u;
      unsigned off = full_off[i];
      if (!full) {  // the last, partial tile: clamp rows past Sk - 1 (finite; masked by the softmax)
        const int row = piece_row(i);
        off = 2u * (unsigned)((min(base + row, Sk - 1) - base) * (i < 2 ? ksd : vsd) + 8 * ((lane % CPR) ^ swz<D>(row)));
      }
      dma_piece(i < 2 ? kt_ : vt_, off, dst);
    }
  };
#pragma unroll
  for (int t = 0; t < NBUF - 1; ++t)
    if (t < ntiles) issue(t);

  // ---- Q, dO fragments (B operands), delta = rowsum(dO * O), LSE ----
  bf16x8 qf[KS], df[KS];
  float dsum = 0.f;
  {
    const int64_t qoff = b * a.q_strides[0] + hq * a.q_strides[2] + (int64_t)qc * a.q_strides[1] + 8 * h;
    const int64_t dooff = b * a.do_strides[0] + hq * a.do_strides[2] + (int64_t)qc * a.do_strides[1] + 8 * h;
    const int64_t ooff = b * a.o_strides[0] + hq * a.o_strides[2] + (int64_t)qc * a.o_strides[1] + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u16x8 qv = *reinterpret_cast<const u16x8*>((const bf16_t*)a.q + qoff + 16 * ks);
      const u16x8 dv = *reinterpret_cast<const u16x8*>((const bf16_t*)a.dout + dooff + 16 * ks);
      const u16x8 ov = *reinterpret_cast<const u16x8*>((const bf16_t*)a.o + ooff + 16 * ks);
      qf[ks] = __builtin_bit_cast(bf16x8, qv);
      df[ks] = __builtin_bit_cast(bf16x8, dv);
#pragma unroll
      for (int j = 0; j < 8; ++j) dsum += bf2f(ov[j]) * bf2f(dv[j]);
    }
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(qf[ks]), "+v"(df[ks]));
  const auto dsw = __builtin_amdgcn_permlane32_swap(__float_as_uint(dsum), __float_as_uint(dsum), false, false);
  const float dall = __uint_as_float(dsw[0]) + __uint_as_float(dsw[1]);
  const bool row_ok = my_q < Sq;
  const float delta = row_ok ? dall : 0.f;
  const float lse2 = row_ok ? a.lse[((int64_t)b * a.heads_q + hq) * Sq + my_q] * LOG2E : INFINITY;
  if (h == 0 && my_q < sq_pad) {  // for attn_bwd_kv_kernel (padding rows: P = 0, delta = 0)
    lse2_g[(int64_t)bh * sq_pad + my_q] = lse2;
    delta_g[(int64_t)bh * sq_pad + my_q] = -delta;
  }
  const float nl2 = -lse2, ndl = -delta;

  // per-lane LDS offsets (pinned: hipcc would otherwise re-derive the swizzles)
  unsigned ro[KS], tro[DT][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) ro[ks] = lds_off<D>(r, 2 * ks + h);
  {
    const int g = lane >> 4, i = lane & 15, hh = g >> 1, qq = i >> 2, p = i & 3;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int col = 32 * dt + 16 * (g & 1) + 4 * p;
      tro[dt][0] = lds_off<D>(4 * hh + qq, col >> 3) + (col & 7) * 2;
      tro[dt][1] = lds_off<D>(4 * hh + qq + 8, col >> 3) + (col & 7) * 2;
    }
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(ro[ks]));
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) asm volatile("" : "+v"(tro[dt][0]), "+v"(tro[dt][1]));

  f32x16 dq[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dq[dt] = (f32x16)0.f;
  // S^T / dP^T of two tiles: set 0 (even tiles) and set 1 (odd tiles)
  f32x16 Sa[2], Pa[2], Sb[2], Pb[2];

  auto slot_base = [&](int tile) __attribute__((always_inline)) {
    return smem + (unsigned)(tile & (NBUF - 1)) * (unsigned)SLOT;
  };
  // M1 MFMA i of a tile into (s, dp): i < 8 S^T (A = K rows), else dP^T (A = V rows)
  auto m1_read = [&](const char* kb, int i) __attribute__((always_inline)) {
    const int kt = (i & 7) >> 2, ks = i & 3;
    return lds_read_b128(kb + (i < 8 ? 0 : IMG), ro[ks] + kt * 32 * RB);
  };
  // plain (compiler-ordered) M1 of one tile: the prologue and the sets' first use
  auto m1_plain = [&](const char* kb, f32x16 (&s)[2], f32x16 (&dp)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      s[kt] = (f32x16)0.f;
      dp[kt] = (f32x16)0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s[kt] = mfma32(m1_read(kb, 4 * kt + ks), qf[ks], s[kt]);
        dp[kt] = mfma32(m1_read(kb, 8 + 4 * kt + ks), df[ks], dp[kt]);
      }
    }
  };
  // causal diagonal / ragged tile: keys past the lane's row (or >= Sk) get S = -inf (P = 0, dS = 0)
  auto mask_tile = [&](f32x16 (&s)[2], int n0) __attribute__((always_inline)) {
    const int rel = lim_lane - n0 - 4 * h;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = 32 * kt + (i & 3) + 8 * (i >> 2);
        s[kt][i] = c <= rel ? s[kt][i] : -INFINITY;
      }
  };
  // tail: P, dS and dQ of the wave's last tile (compiler-ordered)
  auto tail = [&](const char* kb, const f32x16 (&s)[2], const f32x16 (&dp)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        float ds[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          ds[j] = fast_exp2(__builtin_fmaf(s[kt][8 * st + j], scale_log2, nl2)) * (dp[kt][8 * st + j] + ndl);
        const bf16x8 dsf = pack_bf16x8(ds);
        const char* rowb = kb + (32 * kt + 16 * st) * RB;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) dq[dt] = mfma32(tr_pair_q64(rowb, tro[dt][0], tro[dt][1]), dsf, dq[dt]);
      }
  };

  // Interval of tile t: VALU of tile t (set cur) and its dQ MFMAs (K(t) transposed) beside the M1 MFMAs of
  // tile t + 1 (set nxt, K(t + 1) / V(t + 1) rows), in the 24-slot order of bq_slot.
  auto interval = [&](const char* kb_cur, const char* kb_nxt, const f32x16 (&sc)[2], const f32x16 (&pc)[2],
                      f32x16 (&sn)[2], f32x16 (&pn)[2]) __attribute__((always_inline)) {
    float ta[32], e[32], d[32], ds[32];
    unsigned pk[16];
    bf16x8 opnd[24];
    auto read = [&](auto s_tag) __attribute__((always_inline)) {
      constexpr int sl = decltype(s_tag)::value, m = bq_slot(sl);
      if constexpr ((PICO_BQ64_ABL & 1) != 0) {
        opnd[sl] = m < 16 ? qf[m & 3] : df[m & 3];
      } else if constexpr (m < 16) {
        opnd[sl] = m1_read(kb_nxt, m);
      } else {
        constexpr int c = (m - 16) >> 1, dt = (m - 16) & 1, kt = c >> 1, st = c & 1;
        opnd[sl] = tr_pair_q64(kb_cur + (32 * kt + 16 * st) * RB, tro[dt][0], tro[dt][1]);
      }
    };
    auto mfma_slot = [&](auto s_tag) __attribute__((always_inline)) {
      constexpr int sl = decltype(s_tag)::value, m = bq_slot(sl);
      if constexpr ((PICO_BQ64_ABL & 8) != 0 && m < 16) {
        sn[m & 1][m >> 1] += __builtin_bit_cast(float, opnd[sl][0] == opnd[sl][1] ? 1u : 0u);
      } else if constexpr ((PICO_BQ64_ABL & 16) != 0 && m >= 16) {
        dq[m & 1][m & 15] += __builtin_bit_cast(float, opnd[sl][0] == opnd[sl][1] ? pk[(m - 16) & 15] : 0u);
      } else if constexpr (m < 8) {
        constexpr int kt = m >> 2, ks = m & 3;
        sn[kt] = mfma32(opnd[sl], qf[ks], ks == 0 ? (f32x16)0.f : sn[kt]);
      } else if constexpr (m < 16) {
        constexpr int kt = (m - 8) >> 2, ks = (m - 8) & 3;
        pn[kt] = mfma32(opnd[sl], df[ks], ks == 0 ? (f32x16)0.f : pn[kt]);
      } else {
        constexpr int c = (m - 16) >> 1, dt = (m - 16) & 1;
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
        const u32x4 pw = {pk[4 * c], pk[4 * c + 1], pk[4 * c + 2], pk[4 * c + 3]};
        dq[dt] = mfma32(opnd[sl], __builtin_bit_cast(bf16x8, pw), dq[dt]);
      }
    };
    auto valu = [&](auto k_tag) __attribute__((always_inline)) {
      constexpr int k = decltype(k_tag)::value;
      constexpr int c = k / 36, op = bq_op(k % 36);
      constexpr int ty = op / 100, j = op % 100, kt = c >> 1, st = c & 1, q = 8 * c + j;
      typedef __attribute__((ext_vector_type(2))) float f32x2;
      typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
      if constexpr ((PICO_BQ64_ABL & 2) != 0) {
        if constexpr (ty == 4) pk[4 * c + j] = __float_as_uint(sc[kt][8 * st + 2 * j]) ^ __float_as_uint(pc[kt][8 * st + 2 * j + 1]);
      } else if constexpr ((PICO_BQ64_ABL & 64) != 0) {  // independent ops (each result consumed by an empty asm)
        const float src = sc[kt][8 * st + (j & 7)], src2 = pc[kt][8 * st + (j & 7)];
        float rr;
        if constexpr (ty == 0) rr = __builtin_fmaf(src, scale_log2, nl2);
        else if constexpr (ty == 1) rr = fast_exp2(src2);
        else if constexpr (ty == 2) rr = src2 + ndl;
        else if constexpr (ty == 3) rr = src * src2;
        else {
          typedef __attribute__((ext_vector_type(2))) float f32x2;
          typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
          pk[4 * c + j] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){src, src2}, bf16x2));
          rr = 0.f;
        }
        asm volatile("" ::"v"(rr));
      } else if constexpr (ty == 0) ta[q] = __builtin_fmaf(sc[kt][8 * st + j], scale_log2, nl2);
      else if constexpr (ty == 1) e[q] = (PICO_BQ64_ABL & 128) ? ta[q] * 1.0001f : fast_exp2(ta[q]);
      else if constexpr (ty == 2) d[q] = pc[kt][8 * st + j] + ndl;
      else if constexpr (ty == 3) ds[q] = e[q] * d[q];
      else pk[4 * c + j] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){ds[8 * c + 2 * j], ds[8 * c + 2 * j + 1]}, bf16x2));
    };
    static_for<PICO_BQ64_RD>([&](auto s) { read(s); });
    __builtin_amdgcn_sched_barrier(0);
    static_for<24>([&](auto s_) {
      constexpr int sl = decltype(s_)::value;
      mfma_slot(s_);
      constexpr int b0 = bq_first_op(sl), b1 = bq_end_op(sl);
      static_for<b1 - b0>([&](auto j_) { valu(std::integral_constant<int, b0 + decltype(j_)::value>{}); });
      if constexpr (sl + PICO_BQ64_RD < 24) read(std::integral_constant<int, sl + PICO_BQ64_RD>{});
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  // tile t + 1 landed (this wave's pieces; tile t + 2's may stay in flight), then every wave's; every wave
  // is past the interval of t - 1 (the last reader of tile t - 1's slot), which now takes tile t + 3
  auto barrier_dma = [&](int t) __attribute__((always_inline)) {
    if (!(PICO_BQ64_ABL & 4)) {
      if (t + 1 < ntiles) wait_vmcnt(t + 2 < ntiles ? NPW : 0);
      lds_barrier();
    }
    if (!(PICO_BQ64_ABL & 32) && t + NBUF - 1 < ntiles) issue(t + NBUF - 1);
  };

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // prologue tiles and loads landed
  lds_barrier();
  // ---- M1 of tile 0, then intervals 0 .. tl - 1 (pairs: set a -> b, b -> a), the tail of tile tl ----
  m1_plain(slot_base(0), Sa, Pa);
  int t = 0;
  for (; t + 1 < tl; t += 2) {
    barrier_dma(t);
    interval(slot_base(t), slot_base(t + 1), Sa, Pa, Sb, Pb);
    barrier_dma(t + 1);
    interval(slot_base(t + 1), slot_base(t + 2), Sb, Pb, Sa, Pa);
  }
  const bool odd = t < tl;  // one interval left: tile t (set a) -> tile tl (set b)
  if (odd) {
    barrier_dma(t);
    interval(slot_base(t), slot_base(t + 1), Sa, Pa, Sb, Pb);
    ++t;
  }
  // t == tl: the last tile of the wave (a causal diagonal or a ragged end needs the mask)
  barrier_dma(t);
  const bool mask = tl * KT + KT - 1 > lim_first;
  if (odd) {
    if (mask) mask_tile(Sb, tl * KT);
    tail(slot_base(tl), Sb, Pb);
  } else {
    if (mask) mask_tile(Sa, tl * KT);
    tail(slot_base(tl), Sa, Pa);
  }
  for (++t; t < ntiles; ++t) barrier_dma(t);

  // ---- epilogue: lane = query my_q, register i of tile dt = d 32 dt + acc_row(i, h) ----
  if (a.flags & PICO_ATTN_ROPE_BWD) {  // rotate back by -theta: pairs (d, d + D/2) = tiles (dt, dt + DT/2)
    const bf16_t* cp = (const bf16_t*)a.rope_cos + (int64_t)qc * a.rope_stride;
    const bf16_t* sp = (const bf16_t*)a.rope_sin + (int64_t)qc * a.rope_stride;
#pragma unroll
    for (int dt = 0; dt < DT / 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const u16x4 c4 = *reinterpret_cast<const u16x4*>(cp + 32 * dt + 8 * g + 4 * h);
        const u16x4 s4 = *reinterpret_cast<const u16x4*>(sp + 32 * dt + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float cf = bf2f(c4[j]), sf = bf2f(s4[j]);
          const float x1 = dq[dt][4 * g + j], x2 = dq[dt + DT / 2][4 * g + j];
          dq[dt][4 * g + j] = x1 * cf + x2 * sf;
          dq[dt + DT / 2][4 * g + j] = x2 * cf - x1 * sf;
        }
      }
  }
  if (a.flags & PICO_ATTN_DQ_F32_ACCUM) {
    if (!row_ok) return;
    float* dst = (float*)a.dq + b * a.dq_strides[0] + hq * a.dq_strides[2] + (int64_t)my_q * a.dq_strides[1];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float* p = dst + 32 * dt + 8 * g + 4 * h;
#pragma unroll
        for (int j = 0; j < 4; ++j) p[j] += dq[dt][4 * g + j] * scale;
      }
    return;
  }
  bf16_t* dst = (bf16_t*)a.dq + b * a.dq_strides[0] + hq * a.dq_strides[2] + (int64_t)qc * a.dq_strides[1];
  store_row_bf16_x16<DT>(dst, h, row_ok, [&](int dt, int i) { return dq[dt][i] * scale; });
}

}  // namespace

// Launch of the D = 64 pipelined dQ kernel with attn_bwd_q_kernel's arguments (attn_bwd_split.hip decides).
bool pico_attn_bwd_q64_ok(const pico_attn_args* a) {
  return a->head_dim == 64 && a->k_strides[1] * 2 * KT < (1ll << 31) && a->v_strides[1] * 2 * KT < (1ll << 31);
}
int pico_attn_bwd_q64(const pico_attn_args* a, hipStream_t s, float* lse2, float* delta, int sq_pad, int nfront) {
  const float sl2 = a->softmax_scale * LOG2E;
  const int nmb = (int)((a->seqlen_q + QB - 1) / QB);
  const int64_t gq = (int64_t)nmb * a->batch * a->heads_q;
  PICO_REQUIRE(gq < (1ll << 31), "pico_attn_bwd: grid too large");
  if (a->causal) {
    PICO_TRY(pico_launch(PICO_K_ATTN_BWD_Q, "attn_bwd_q", attn_bwd_q64_kernel<true>, dim3((int)gq), dim3(256), 0, s, *a,
                         a->softmax_scale, sl2, lse2, delta, sq_pad, nfront));
  } else {
    PICO_TRY(pico_launch(PICO_K_ATTN_BWD_Q, "attn_bwd_q", attn_bwd_q64_kernel<false>, dim3((int)gq), dim3(256), 0, s, *a,
                         a->softmax_scale, sl2, lse2, delta, sq_pad, nfront));
  }
  return 0;
}
