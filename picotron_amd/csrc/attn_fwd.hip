// Flash-attention forward for gfx950: causal / non-causal, GQA, bf16 MFMA, fp32 online softmax,
// fp32 LSE output.
//
// Replaces flash_attn_func(q, k, v, causal=True) (ref picotron/model.py:32-36,153; eager oracle
// F.scaled_dot_product_attention :156) and the ring block forward ring_attention_forward
// (ref picotron/context_parallel/context_parallel.py:112-128), which additionally returns the LSE.
//
// Structure (one workgroup = 4 waves = 128 query rows of one (batch, q-head); 64-key tiles):
//   * Q stays in registers for the whole sweep (B operand, 8 bf16 per lane per 16-wide k-step).
//   * K and V tiles arrive by LDS-DMA (global_load_lds_dwordx4, the swizzle applied to the per-lane source
//     address) into an NBUF-slot ring of conflict-free LDS images, prefetch distance NBUF - 1 (below).
//   * Swapped product S^T = K * Q^T (v_mfma_f32_32x32x16_bf16): the accumulator has the query on
//     the lane and 16 keys in registers, so the online softmax is lane-local (one permlane32 swap
//     for the row max) and P^T is already the B operand of O^T += V^T * P^T (no LDS round trip);
//     V^T fragments come from ds_read_b64_tr_b16 on the row-major V image.
//   * The softmax is written for the VALU budget, which (not the MFMA) bounds D = 64: raw scores
//     are kept unscaled and one FMA per score folds scale*log2(e) and the running max into the
//     exp2 argument; the row sum stays a per-lane partial until the epilogue; O is rescaled only
//     when some row's max grew (wave-uniform vote; exact, no threshold); masking (causal diagonal,
//     key padding) is a separate branch-free body used only on the tiles that need it.
//   * Causal: tiles beyond the diagonal are never loaded; waves skip tiles entirely above their rows;
//     workgroups are issued heaviest-first over all heads (LPT order), and the q-blocks of one head
//     sit nbh (a multiple of 8) block ids apart, i.e. on one XCD, sharing its L2 for K/V.
// FLOPs per (b, h): 4 * Sq * Sk * D (halved by the causal mask).
#include <type_traits>

#include "attn_common.h"

// Build-time variants (A/B measurement only; the shipped defaults are the measured-best):
//   PICO_FWD_RESCALE_THR: rescale O only when a row max grows by more than THR (log2 units; 0 =
//     rescale on every growth). > 0 (cdna_hip_programming.md T13) lets P reach 2^THR: l and O stay
//     exact in fp32 and P is bf16-rounded with the same relative precision as any P <= 1; the final
//     1/l normalisation is unchanged. Measured: THR = 8 -2.7 % (D=64) / -4 % (D=128) kernel time.
//   PICO_FWD_EARLY_V: issue the V^T transposed reads before the softmax VALU (1), after it (0), or
//     by head_dim (-1: early for D = 128 only, where it measured -2.5 %; neutral at D = 64).
#ifndef PICO_FWD_RESCALE_THR
#define PICO_FWD_RESCALE_THR 8
#endif
#ifndef PICO_FWD_EARLY_V
#define PICO_FWD_EARLY_V -1
#endif
// (Measured and dropped: the row sums out of the matrix pipe -- one v_mfma_f32_16x16x32_bf16 of a 0/1
// operand with the packed P^T per 16-key half instead of 32 v_add_f32 per tile -- +2..4 % at D = 64; the
// mask as the C operand of the first S MFMA -- spills at 128 VGPRs; no row max on the common path (P against
// the running max, accepted when every lane's partial sum stays <= 2^THR, else S recomputed max-first) --
// +16 % at C2 although the fallback never ran: the retry loop costs the compiler's schedule more than the 16
// max3 it removes.)

//   PICO_FWD_NBUF_D64 / PICO_FWD_WPE_D64: ring slots and waves per SIMD for D = 64. 2 / 4 (shipped):
//     four 32-KiB workgroups per CU, prefetch distance 1, 128 VGPRs without spills; 3 / 3: three
//     48-KiB workgroups per CU. Measured C2 causal 36.0 -> 34.8 us, full 54.9 -> 52.5, GQA 33.5 -> 32.3.
// PICO_FWD_WGSTAMP: diagnostic build -- every workgroup records s_memrealtime (100 MHz, chip-wide) at entry,
// loop start, loop end and after its stores drained, into a.workspace (4 x 8 B per workgroup, if non-null)
#ifndef PICO_FWD_WGSTAMP
#define PICO_FWD_WGSTAMP 0
#endif
// PICO_FWD_SNAKE: causal block order. The grid is dispatched in rounds of one workgroup per CU; when every
// workgroup is resident at once (C2: 1024 = 4 per CU) each CU keeps the blocks one round hands it, so a
// plain heaviest-first order gives the CUs that take the heaviest block of every round 40 tiles and the
// others 32. Odd rounds run lightest-first instead (a snake over the sorted list): 36 tiles on every CU.
#ifndef PICO_FWD_SNAKE
#define PICO_FWD_SNAKE 1
#endif

#ifndef PICO_FWD_NBUF_D64
#define PICO_FWD_NBUF_D64 2
#endif
#ifndef PICO_FWD_WPE_D64
#define PICO_FWD_WPE_D64 4
#endif

namespace {

constexpr int BM = 128;  // query rows per workgroup (32 per wave)
constexpr int BN = 64;   // keys per tile

// LDS images (one set per ring slot), chosen so that every read of a tile is one per-lane base
// register plus compile-time immediates, and conflict-free:
//   K: KS images [64 keys][16 d] (32-B rows), 16-B chunk h of row `key` stored at chunk h ^ bit3(key):
//      a ds_read_b128 lane group (16 rows, one chunk) covers all 64 banks exactly once;
//   V: D/32 images [64 keys][32 d] (64-B rows), unswizzled: each 32-lane half of a ds_read_b64_tr_b16
//      reads 4 consecutive rows x 64 B = 256 contiguous bytes.
// Tiles arrive by LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave-instruction, lane-linear in LDS),
// so the swizzle is applied to the per-lane SOURCE address. NBUF-slot ring, prefetch distance NBUF-1.
template <int D>
struct FwdCfg {
  static constexpr int KS = D / 16, DT = D / 32;
  static constexpr int KIMG = BN * 32;                  // bytes per 16-wide K image
  static constexpr int VIMG = BN * 64;                  // bytes per 32-wide V image
  static constexpr int SLOT = 2 * BN * D * 2;           // K + V of one tile
  static constexpr int NBUF = D == 64 ? PICO_FWD_NBUF_D64 : 2;  // LDS: 16 KiB (D=64) / 32 KiB (D=128) per slot
  static constexpr int NI = 2 * KS + 4 * DT;            // 1-KiB DMA pieces per tile
  static constexpr int NIW = NI / 4;                    // ... per wave
  static constexpr int WAVES_PER_EU = D == 64 ? PICO_FWD_WPE_D64 : 2;
};

// max over both lane halves (lane r and r + 32 hold the same query row)
PICO_DEV float halves_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
PICO_DEV float halves_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, FwdCfg<D>::WAVES_PER_EU)
__attribute__((amdgpu_waves_per_eu(FwdCfg<D>::WAVES_PER_EU, FwdCfg<D>::WAVES_PER_EU))) void attn_fwd_kernel(const pico_attn_args a, float scale_log2, int round_len) {
  using C = FwdCfg<D>;
  constexpr bool EARLY_V = PICO_FWD_EARLY_V < 0 ? D == 128 : PICO_FWD_EARLY_V != 0;
  constexpr int KS = C::KS;  // k-steps of the S^T product
  constexpr int DT = C::DT;  // 32-wide output tiles of O^T
  __shared__ __attribute__((aligned(16))) char smem[C::NBUF * C::SLOT];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (scalar branches)
  const int r = lane & 31, h = lane >> 5;
#if PICO_FWD_WGSTAMP
  unsigned long long wgs[4];
  wgs[0] = __builtin_amdgcn_s_memrealtime();
#endif

  // LPT order: heaviest query blocks of every head first (snaked per dispatch round, PICO_FWD_SNAKE).
  const int nmb = (int)((a.seqlen_q + BM - 1) / BM);
  const int nbh = (int)(a.batch * a.heads_q);
  int lin = blockIdx.x;
  if (PICO_FWD_SNAKE && CAUSAL) {  // reversed in groups of 8 (blockIdx % 8 = the XCD stays lin % 8: the
    // blocks of one head keep sharing one XCD's L2); full rounds only
    const int rnd = lin / round_len, pos = lin - rnd * round_len;
    if ((rnd & 1) && (rnd + 1) * round_len <= (int)gridDim.x) lin = rnd * round_len + (round_len - 8 - (pos & ~7)) + (pos & 7);
  }
  const int mb = CAUSAL ? (nmb - 1 - lin / nbh) : (lin / nbh);
  const int bh = lin % nbh;
  const int b = bh / (int)a.heads_q;
  const int hq = bh % (int)a.heads_q;
  const int hk = hq / (int)(a.heads_q / a.heads_kv);
  const int Sq = (int)a.seqlen_q, Sk = (int)a.seqlen_k;

  const bf16_t* qg = (const bf16_t*)a.q + b * a.q_strides[0] + hq * a.q_strides[2];
  const bf16_t* kg = (const bf16_t*)a.k + b * a.k_strides[0] + hk * a.k_strides[2];
  const bf16_t* vg = (const bf16_t*)a.v + b * a.v_strides[0] + hk * a.v_strides[2];
  const int64_t ksd = a.k_strides[1], vsd = a.v_strides[1];

  const int q0 = mb * BM;
  const int qw = q0 + wave * 32;  // this wave's first query row
  const int my_q = qw + r;

  // ---- Q fragments (B operand of S^T = K Q^T): Q[my_q][16 ks + 8 h + j] ----
  bf16x8 qf[KS];
  {
    const bf16_t* qp = qg + (int64_t)min(my_q, Sq - 1) * a.q_strides[1] + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(qp + 16 * ks));
  }
  // PICO_ATTN_ROPE_Q_FWD: q holds the unrotated rows. The rotate-half pairs (d, d + D/2) sit in the
  // same lane (k-steps ks and ks + KS/2), so the rotation happens in registers, with the rope
  // kernel's arithmetic (fp32, one rounding). The tables load beside q; the rotation runs after the
  // first K/V tiles are issued, and the rotated row (still in qf) is stored to dq in the epilogue, so
  // neither sits in the vmcnt queue ahead of the first tiles. Each query row is loaded by exactly one
  // lane of one workgroup, so dq may alias q.
  const bool rope_q = (a.flags & PICO_ATTN_ROPE_Q_FWD) != 0;
  u16x8 rc[KS / 2], rs[KS / 2];
  if (rope_q) {
    const int pos = min(my_q, Sq - 1);
    const bf16_t* cp = (const bf16_t*)a.rope_cos + (int64_t)pos * a.rope_stride + 8 * h;
    const bf16_t* sp = (const bf16_t*)a.rope_sin + (int64_t)pos * a.rope_stride + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS / 2; ++ks) {
      rc[ks] = *reinterpret_cast<const u16x8*>(cp + 16 * ks);
      rs[ks] = *reinterpret_cast<const u16x8*>(sp + 16 * ks);
    }
  }

  // tiles this workgroup visits; the last key any of its rows may see is `wg_lim`
  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + BM);
  const int ntiles = (kend + BN - 1) / BN;
  // the wave's rows see keys <= lim_w (last row); tiles entirely <= first_lim need no mask
  const int lim_last = CAUSAL ? min(qw + 31, Sk - 1) : Sk - 1;
  const int lim_first = CAUSAL ? min(qw, Sk - 1) : Sk - 1;
  const int lim_lane = CAUSAL ? min(my_q, Sk - 1) : Sk - 1;  // this lane's row: keys <= lim_lane

  // ---- LDS-DMA staging: piece j (wave w issues j = w, w + 4, ...) ----
  // K piece (j < 2 KS): image ks = j / 2, rows 32 (j & 1) + lane / 2, LDS chunk lane & 1, which holds
  // source chunk h = (lane & 1) ^ bit3(row). V piece: image dt, rows 16 p + lane / 4, 16-B part lane & 3.
  // Per piece: this lane's source row within the tile and element column; LDS destination offset.
  // K and V pieces are uniform per (wave, i), so the K/V choice is a scalar select.
  int src_row[C::NIW], src_col[C::NIW];
  unsigned dst_off[C::NIW];
  bool is_k[C::NIW];
#pragma unroll
  for (int i = 0; i < C::NIW; ++i) {
    const int j = wave + 4 * i;
    if (j < 2 * KS) {
      const int ks = j >> 1, row = 32 * (j & 1) + (lane >> 1);
      src_row[i] = row;
      src_col[i] = 16 * ks + 8 * ((lane & 1) ^ ((row >> 3) & 1));
      dst_off[i] = ks * C::KIMG + 32 * (j & 1) * 32;
      is_k[i] = true;
    } else {
      const int jv = j - 2 * KS, dt = jv >> 2, row = 16 * (jv & 3) + (lane >> 2);
      src_row[i] = row;
      src_col[i] = 32 * dt + 8 * (lane & 3);
      dst_off[i] = BN * D * 2 + dt * C::VIMG + 16 * (jv & 3) * 64;
      is_k[i] = false;
    }
  }
  // element offsets within a tile for full tiles (rows never clamped)
  unsigned src_off_b[C::NIW];
#pragma unroll
  for (int i = 0; i < C::NIW; ++i) src_off_b[i] = (unsigned)(src_row[i] * (is_k[i] ? ksd : vsd) + src_col[i]) * 2u;
  const char* const kbase = (const char*)kg;
  const char* const vbase = (const char*)vg;
  const int64_t kst = (int64_t)BN * ksd * 2, vst = (int64_t)BN * vsd * 2;  // bytes per tile
  const unsigned smem_lds0 = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr(smem));
  auto issue = [&](int tile) __attribute__((always_inline)) {
    char* slot = smem + (unsigned)(tile % C::NBUF) * (unsigned)C::SLOT;
    const int base = tile * BN;
    if (base + BN <= Sk) {
      const unsigned sl = smem_lds0 + (unsigned)(tile % C::NBUF) * (unsigned)C::SLOT;
#pragma unroll
      for (int i = 0; i < C::NIW; ++i)
        dma_piece(is_k[i] ? kbase + tile * kst : vbase + tile * vst, src_off_b[i], sl + dst_off[i]);
    } else {  // last, partial tile
      int ln;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
#pragma unroll
      for (int i = 0; i < C::NIW; ++i) {
        const int j = wave + 4 * i;
        int row, col;
        if (j < 2 * KS) {
          row = 32 * (j & 1) + (ln >> 1);
          col = 16 * (j >> 1) + 8 * ((ln & 1) ^ ((row >> 3) & 1));
        } else {
          const int jv = j - 2 * KS;
          row = 16 * (jv & 3) + (ln >> 2);
          col = 32 * (jv >> 2) + 8 * (ln & 3);
        }
        const int key = min(base + row, Sk - 1);
        const bf16_t* src = is_k[i] ? kg + (int64_t)key * ksd + col : vg + (int64_t)key * vsd + col;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(slot + dst_off[i]),
                                         16, 0, 0);
      }
    }
  };

  // per-lane LDS read offsets (everything else is an immediate)
  const unsigned smem_lds = lds_addr(smem);
  const unsigned k_lane = r * 32 + 16 * (h ^ ((r >> 3) & 1));
  const unsigned v_lane = (4 * h + ((lane & 15) >> 2)) * 64 + 32 * ((lane >> 4) & 1) + 8 * (lane & 3);

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x16)0.f;
  float m_i = -INFINITY, neg_m = 0.f, thr_raw = -INFINITY;
  const float inv_sl2 = 1.f / scale_log2;
  float l_i = 0.f;        // per-lane partial row sum (this lane's keys only)

  // V^T operands for keys 32 kt .. 32 kt + 31 of the tile (2 st x DT, inline-asm transposed reads)
  auto v_reads = [&](bf16x8 (&vf)[2][DT], unsigned va, auto kt_tag) __attribute__((always_inline)) {
    constexpr int KT = decltype(kt_tag)::value;
    static_for<2>([&](auto st_) {
      constexpr int ST = decltype(st_)::value;
      static_for<DT>([&](auto dt_) {
        constexpr int DTI = decltype(dt_)::value;
        vf[ST][DTI] = tr_operand_imm<BN * D * 2 + DTI * C::VIMG + (32 * KT + 16 * ST) * 64, 8 * 64>(va);
      });
    });
  };
  // P^T (keys 32 kt .. 32 kt + 31 of the tile) times V: 2 * DT MFMAs.
  auto pv_mfma = [&](const f32x16& p, const bf16x8 (&vf)[2][DT]) __attribute__((always_inline)) {
    float pv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) pv[j] = p[j];
    const bf16x8 pf0 = pack_bf16x8(pv), pf1 = pack_bf16x8(pv + 8);  // one v_cvt_pk_bf16_f32 per pair
    lds_wait_all();
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] = mfma32(vf[0][dt], pf0, o[dt]);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] = mfma32(vf[1][dt], pf1, o[dt]);
  };

  // S^T of one 64-key tile (2 x 16 accumulators), masked when MASK
  auto compute_s = [&](const char* kb, int n0, bool mask, f32x16 (&s)[2]) __attribute__((always_inline)) {
    // every K fragment of the tile requested before the first MFMA (one LDS latency per tile, not per step)
    bf16x8 kf[2][KS];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) kf[kt][ks] = lds_read_b128(kb, ks * C::KIMG + kt * 32 * 32);
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      s[kt] = (f32x16)0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) s[kt] = mfma32(kf[kt][ks], qf[ks], s[kt]);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 2 * KS, 0);  // the K reads first,
    __builtin_amdgcn_sched_group_barrier(0x008, 2 * KS, 0);  // then the S MFMAs
    // lane holds row my_q, keys n0 + 32 kt + acc_row(i, h) = n0 + 4h + c(kt, i)
    if (mask) {  // wave-uniform
      const int rel = lim_lane - n0 - 4 * h;  // key allowed iff c <= rel
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int c = 32 * kt + (i & 3) + 8 * (i >> 2);
          s[kt][i] = c <= rel ? s[kt][i] : -INFINITY;
        }
    }
  };

  // One 64-key tile for this wave. MASK: apply key <= lim_lane (causal) and key < Sk.
  auto tile_body = [&](const char* kb, unsigned vaddr, int n0, bool mask) __attribute__((always_inline)) {
    f32x16 s[2];
    compute_s(kb, n0, mask, s);
    bf16x8 vf0[2][DT], vf1[2][DT];
    if constexpr (EARLY_V) {  // in flight during the softmax VALU below
      v_reads(vf0, vaddr, std::integral_constant<int, 0>{});
      v_reads(vf1, vaddr, std::integral_constant<int, 1>{});
    }
    float mx = s[0][0];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = (kt == 0 ? 1 : 0); i < 16; ++i) mx = fmaxf(mx, s[kt][i]);
    if (__builtin_amdgcn_ballot_w64(mx > thr_raw)) {
      const float m_tile = halves_max(mx) * scale_log2;
      const float m_new = fmaxf(m_i, m_tile);
      const float alpha = m_i == -INFINITY ? 0.f : fast_exp2(m_i - m_new);
      l_i *= alpha;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      m_i = m_new;
      neg_m = m_i == -INFINITY ? 0.f : -m_i;
      thr_raw = (m_i + (float)PICO_FWD_RESCALE_THR) * inv_sl2;
    }
    float lsum0 = 0.f, lsum1 = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const float p0 = fast_exp2(__builtin_fmaf(s[kt][i], scale_log2, neg_m));
        const float p1 = fast_exp2(__builtin_fmaf(s[kt][i + 1], scale_log2, neg_m));
        s[kt][i] = p0;
        s[kt][i + 1] = p1;
        lsum0 += p0;
        lsum1 += p1;
      }
    l_i += lsum0 + lsum1;
    // O^T[dt] += V^T * P^T : A = V^T via transposed LDS reads (per kt: 2 st x DT operands, issued
    // together, one wait), B = packed P^T registers
    if constexpr (!EARLY_V) {
      v_reads(vf0, vaddr, std::integral_constant<int, 0>{});
      pv_mfma(s[0], vf0);
      v_reads(vf1, vaddr, std::integral_constant<int, 1>{});
      pv_mfma(s[1], vf1);
    } else {
      pv_mfma(s[0], vf0);
      pv_mfma(s[1], vf1);
    }
  };

  constexpr int P = C::NBUF - 1;  // prefetch distance
#pragma unroll
  for (int t = 0; t < P; ++t)
    if (t < ntiles) issue(t);
  if (rope_q) {
#pragma unroll
    for (int ks = 0; ks < KS / 2; ++ks) {
      const u16x8 x1 = __builtin_bit_cast(u16x8, qf[ks]), x2 = __builtin_bit_cast(u16x8, qf[ks + KS / 2]);
      u16x8 o1, o2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xa = bf2f(x1[j]), xb = bf2f(x2[j]);
        const float cf = bf2f(rc[ks][j]), sf = bf2f(rs[ks][j]);
        // both products rounded before the sum (no FMA contraction): the rope kernel's and the oracle's
        // fp32 arithmetic bit for bit, so q rotated here == pico_rope's q
        o1[j] = f2bf(__fmul_rn(xa, cf) - __fmul_rn(xb, sf));
        o2[j] = f2bf(__fmul_rn(xb, cf) + __fmul_rn(xa, sf));
      }
      qf[ks] = __builtin_bit_cast(bf16x8, o1);
      qf[ks + KS / 2] = __builtin_bit_cast(bf16x8, o2);
    }
  }

#if PICO_FWD_WGSTAMP
  wgs[1] = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
#endif
  // unrolled by the ring depth: every ring slot is a compile-time offset in the LDS reads
  for (int t0 = 0; t0 < ntiles; t0 += C::NBUF) {
#pragma unroll
    for (int u = 0; u < C::NBUF; ++u) {
      const int t = t0 + u;
      if (t >= ntiles) break;
      // tile t's pieces landed (this wave's), then every wave's (barrier); later tiles stay in flight
      if (P == 2 && t + 1 < ntiles) {
        if constexpr (C::NIW == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      // slot (t + P) % NBUF was last read in iteration t - 1, which every wave has finished
      if (t + P < ntiles) issue(t + P);
      const int n0 = t * BN;
      // wave-uniform: skip (tile above every row), full (every key visible to every row), or masked
      if (n0 <= lim_last) {
        const unsigned slot = (unsigned)u * (unsigned)C::SLOT;
        const char* kb = smem + (slot + k_lane);
        tile_body(kb, smem_lds + slot + v_lane, n0, n0 + BN - 1 > lim_first);
      }
    }
  }

#if PICO_FWD_WGSTAMP
  wgs[2] = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
#endif
  // ---- epilogue: O = O^T / l, LSE = (m + log2 l) * ln2 ----
  // Every lane stays (the 16-byte O stores exchange half-chunks between lanes l and l + 32; only rows
  // < Sq store). O^T (for the out-projection's wgrad) is staged transposed in the now idle LDS ring,
  // [D][BM + 8], and leaves as 16-byte segments of 8 tokens (instead of 2-byte stores per element).
  const float l_tot = halves_sum(l_i);
  const bool row_ok = my_q < Sq;
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  {
    bf16_t* op = (bf16_t*)a.o + b * a.o_strides[0] + hq * a.o_strides[2] + (int64_t)min(my_q, Sq - 1) * a.o_strides[1];
    store_row_bf16_x16<DT>(op, h, row_ok, [&](int dt, int i) { return o[dt][i] * inv; });
  }
  if (rope_q && row_ok) {  // the rotated q row, for the backward
    bf16_t* rq = (bf16_t*)a.dq + b * a.dq_strides[0] + hq * a.dq_strides[2] + (int64_t)my_q * a.dq_strides[1] + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) *reinterpret_cast<u16x8*>(rq + 16 * ks) = __builtin_bit_cast(u16x8, qf[ks]);
  }
  if (a.o_t) {  // uniform: O^T [Hq*D][tokens]
    constexpr int TP = BM + 8;  // pitch (elements) of the transposed staging tile
    static_assert(D * TP * 2 <= C::NBUF * C::SLOT, "O^T staging tile must fit the ring");
    unsigned short* tt = reinterpret_cast<unsigned short*>(smem);
    __syncthreads();  // every wave is past its last ring read
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int d = 32 * dt + 8 * (i >> 2) + 4 * h + (i & 3);
        tt[d * TP + 32 * wave + r] = f2bf(o[dt][i] * inv);
      }
    __syncthreads();
    bf16_t* otb = (bf16_t*)a.o_t + (int64_t)hq * D * a.o_t_ld + (int64_t)b * Sq;
    const bool vec = ((a.o_t_ld | (int64_t)Sq | (int64_t)(uintptr_t)a.o_t) & 7) == 0;
    for (int seg = threadIdx.x; seg < D * BM / 8; seg += 256) {
      const int d = seg / (BM / 8), t8 = seg % (BM / 8);
      const int tok0 = q0 + 8 * t8;
      bf16_t* dst = otb + (int64_t)d * a.o_t_ld + tok0;
      const unsigned short* src = tt + d * TP + 8 * t8;
      if (vec && tok0 + 8 <= Sq) {
        *reinterpret_cast<u16x8*>(dst) = *reinterpret_cast<const u16x8*>(src);
      } else {
        for (int j = 0; j < 8 && tok0 + j < Sq; ++j) dst[j] = src[j];
      }
    }
  }
  if (h == 0 && row_ok) {
    const float lse = l_tot > 0.f ? (m_i + __log2f(l_tot)) * LN2 : -INFINITY;
    a.lse[((int64_t)b * a.heads_q + hq) * Sq + my_q] = lse;
  }
#if PICO_FWD_WGSTAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  wgs[3] = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  if (a.workspace && wave == 0 && lane < 4) ((unsigned long long*)a.workspace)[blockIdx.x * 4 + lane] = wgs[lane & 3];
#endif
}

template <int D>
int launch_fwd(const pico_attn_args* a, hipStream_t s) {
  const int nmb = (int)((a->seqlen_q + BM - 1) / BM);
  const int64_t nblk = (int64_t)nmb * a->batch * a->heads_q;
  PICO_REQUIRE(nblk < (1ll << 31), "pico_attn_fwd: grid too large");
  const float sl2 = a->softmax_scale * LOG2E;
  PICO_REQUIRE(sl2 > 0.f, "pico_attn_fwd: softmax_scale must be positive");
  const int rl = pico_num_cus() / 8 * 8 > 0 ? pico_num_cus() / 8 * 8 : 8;  // snake rounds: whole XCD groups
  if (a->causal) {
    PICO_TRY(pico_launch(PICO_K_ATTN_FWD, "attn_fwd", attn_fwd_kernel<D, true>, dim3((int)nblk), dim3(256), 0, s, *a, sl2, rl));
  } else {
    PICO_TRY(pico_launch(PICO_K_ATTN_FWD, "attn_fwd", attn_fwd_kernel<D, false>, dim3((int)nblk), dim3(256), 0, s, *a, sl2, rl));
  }
  return 0;
}

}  // namespace

int pico_attn_check_common(const pico_attn_args* a, const char* op);
int pico_attn_fwdp(const pico_attn_args* a, hipStream_t s);
extern "C" int pico_attn_fwd(const pico_attn_args* a, void* stream) {
  int rc = pico_attn_check_common(a, "pico_attn_fwd");
  if (rc) return rc;
  PICO_REQUIRE(a->o && a->lse, "pico_attn_fwd: null output");
  PICO_REQUIRE(!a->o_t || a->o_t_ld >= a->batch * a->seqlen_q, "pico_attn_fwd: o_t_ld must cover the tokens");
  if (a->flags & PICO_ATTN_ROPE_Q_FWD) {
    PICO_REQUIRE(a->dq && a->rope_cos && a->rope_sin, "pico_attn_fwd: ROPE_Q_FWD needs dq and the cos/sin tables");
    PICO_REQUIRE(((uintptr_t)a->dq | (uintptr_t)a->rope_cos | (uintptr_t)a->rope_sin) % 16 == 0,
                 "pico_attn_fwd: ROPE_Q_FWD needs 16-byte aligned dq and tables");
    PICO_REQUIRE(a->rope_stride % 8 == 0 && a->rope_stride >= a->head_dim / 2,
                 "pico_attn_fwd: bad rope table row stride %lld", (long long)a->rope_stride);
    for (int d = 0; d < 3; ++d)
      PICO_REQUIRE(a->dq_strides[d] % 8 == 0, "pico_attn_fwd: dq strides must be multiples of 8 elements");
  }
  if (a->batch == 0 || a->seqlen_q == 0 || a->heads_q == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int rp = pico_attn_fwdp(a, s);  // the persistent 64-row-per-wave kernel where it applies (attn_fwdp.hip)
  if (rp >= 0) return rp;
  if (a->head_dim == 64) return launch_fwd<64>(a, s);
  return launch_fwd<128>(a, s);
}
