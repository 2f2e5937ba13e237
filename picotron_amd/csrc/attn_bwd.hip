// Flash-attention backward for gfx950: dQ, dK, dV from (Q, K, V, O, dO, LSE); causal / non-causal,
// GQA, bf16 MFMA with fp32 accumulation.
//
// Replaces flash-attn's backward of flash_attn_func (ref picotron/model.py:36) and the ring block
// backward ring_attention_backward (ref picotron/context_parallel/context_parallel.py:130-155),
// which recomputes P from the (global) O and LSE:  P = exp(scale*QK^T - LSE), dV = P^T dO,
// dP = dO V^T, delta = rowsum(dO * O), dS = P * (dP - delta), dQ = scale * dS K, dK = scale * dS^T Q.
//
// attn_bwd_pre_kernel: delta and LSE*log2(e) into [B*Hq][Sq_pad] fp32 arrays (padding rows get
// LSE = +inf, delta = 0, so padded query rows contribute P = dS = 0 without any masking).
// attn_bwd_kernel: one workgroup = 8 waves = 256 keys of one (batch, kv-head); wave w owns keys
// 32w..32w+31 with the key on the MFMA lane and keeps dK^T/dV^T of its keys in accumulators for the
// whole sweep over (q-heads of the group) x (32-row query tiles), so dK/dV need no cross-workgroup
// sum. Per tile:
//   * Q, dO (XOR-swizzled row-major images serving both row and transposed reads) and the tile's
//     LSE/delta arrive by LDS-DMA (global_load_lds_dwordx4) into a 3-slot ring, two tiles ahead, so
//     HBM/L2 latency hides under two tiles of compute; one barrier opens each tile;
//   * S, dP (MFMA, key on the lane) -> P, dS (VALU) -> dV += P^T dO, dK += dS^T Q (MFMA; the dO / Q
//     operand read transposed with ds_read_b64_tr_b16);
//   * dS crosses LDS once as a [key][q] image written with 4 ds_write_b64 per lane, then
//     dQ partial = dS K over the block's keys (16x16x32 MFMAs, both operands by transposed reads)
//     is stored in fp32 to this key block's slab; attn_bwd_dq_kernel sums the slabs in key-block
//     order (no atomics: plain stores run ~4-5x the chip's float-atomic rate, and the result is
//     bitwise reproducible).
// FLOPs per (b, h): 10 * Sq * Sk * D (halved by the causal mask); 2.5x the forward.
#include "attn_common.h"

// Build-time variants (A/B measurement only; the shipped defaults are the measured-best):
//   PICO_BWD_WAVES_PER_EU_D64: register budget for D = 64 (2: <= 256 VGPRs, one 512-thread workgroup
//     per CU; 4: <= 128 VGPRs, two per CU — their LDS (75 KiB each) fits)
#ifndef PICO_BWD_WAVES_PER_EU_D64
#define PICO_BWD_WAVES_PER_EU_D64 2
#endif
//   PICO_BWD_STAMP: diagnostic build — workgroup 0 records s_memtime stamps per (wave, tile, phase) in LDS
//     and dumps them after the trash slot (workspace grows by STAMP_BYTES); results unchanged
#ifndef PICO_BWD_STAMP
#define PICO_BWD_STAMP 0
#endif
//   PICO_BWD_SCHED: S/dP operand reads all issued before the MFMAs (sched_group_barrier) (1) or
//     left to the scheduler (0)
#ifndef PICO_BWD_SCHED
#define PICO_BWD_SCHED 1
#endif
//   PICO_BWD_STAGGER: waves 4-7 run the dQ tile of t-1 BEFORE tile t's S/dP (1) or after (0)
#ifndef PICO_BWD_STAGGER
#define PICO_BWD_STAGGER 1
#endif
//   PICO_BWD_GROUP_D64: query tiles per workgroup barrier for D = 64 (the ring holds two groups; 2G dS^T
//     images). D = 128 keeps 1 (its LDS has no room for more dS images)
#ifndef PICO_BWD_GROUP_D64
#define PICO_BWD_GROUP_D64 2
#endif
//   PICO_BWD_GROUP_UNROLL: unroll factor of the loop over a group's tiles (1: one copy of the tile code)
#ifndef PICO_BWD_GROUP_UNROLL
#define PICO_BWD_GROUP_UNROLL 1
#endif

namespace {

constexpr int BK = 256;  // keys per workgroup (128 with two workgroups per CU measured slower: 93 -> 100 us)
constexpr int STAMP_TILES = 40, STAMP_PH = 6;
constexpr int64_t STAMP_BYTES = PICO_BWD_STAMP ? 8 * STAMP_TILES * STAMP_PH * 8 : 0;
constexpr int BQ = 32;   // query rows per tile

template <int D>
struct BwdCfg {
  static constexpr int NW = BK / 32;  // waves (32 keys each)
  static constexpr int NTH = NW * 64;
  static constexpr int KS = D / 16, DT = D / 32, CPR = D / 8;
  static constexpr int RB = D * 2;              // bytes per Q/dO/K image row
  static constexpr int QIMG = BQ * RB;          // one Q (or dO) tile image
  static constexpr int LSD = 1024;              // LSE*log2e [32] | delta [32] (one DMA piece)
  static constexpr int SLOT = 2 * QIMG + LSD;
  static constexpr int KIMG = BK * RB;
  static constexpr int DSIMG = BK * BQ * 2;     // dS^T [key][q] bf16, 64-B rows (2G: this group's, the last)
  static constexpr int G = D == 64 ? PICO_BWD_GROUP_D64 : 1;  // tiles per barrier
  static constexpr int NBUF = D == 64 ? 4 : 3;  // ring slots
  static constexpr int PD = NBUF - G;           // prefetch distance (tiles)
  static constexpr int SMEM = KIMG + NBUF * SLOT + 2 * G * DSIMG;
  static_assert(PD >= 1, "ring too small for the group");
  static constexpr int RPP = 1024 / RB;         // image rows per 1-KiB DMA piece
  static constexpr int NQP = QIMG / 1024;       // pieces per Q (or dO) tile
  static constexpr int NP = 2 * NQP + 1;        // pieces per tile
  static constexpr int NPW = (NP + NW - 1) / NW;  // max pieces per wave
};

// byte offset of column q of key row `key` in the dS^T image [key][q] (64-B rows of eight 8-B pieces,
// piece index XOR (key >> 1) & 7): the 4 x ds_write_b64 per lane (16 consecutive keys, one piece) and
// the transposed reads of the dQ A operand are both bank-conflict free (scripts/lds_conflicts.py;
// the previous half-swap layout made the writes 4-way)
PICO_DEV int ds_img_off(int key, int q) {
  return key * 64 + 8 * ((q >> 2) ^ ((key >> 1) & 7)) + 2 * (q & 3);
}

// K block image [256 keys][D]: 16-B chunk index XOR a linear function of row bits 0-3, found by
// exhaustive search (scripts/lds_conflicts.py) so that both uses are conflict free: the ds_read_b128
// row reads of the S operand (rows 32w + r) and the ds_read_b64_tr_b16 reads of the dQ operand
// (rows kk + 8g + q, 16-column blocks). The Q/dO layout lds_off<D> was 2-way on the latter.
template <int D>
PICO_DEV int kswz(int row) {
  if constexpr (D == 64)
    return (((row >> 1) & 1) << 1) ^ ((row >> 2) & 1) ^ (((row >> 3) & 1) << 2);
  return ((row & 1) << 1) ^ (((row >> 1) & 1) << 2) ^ ((row >> 2) & 1) ^ (((row >> 3) & 1) << 3);
}
template <int D>
PICO_DEV int kimg_off(int row, int chunk) {
  return row * (D * 2) + 16 * (chunk ^ kswz<D>(row));
}
// 16x16x32 B operand K[k = row0 + 8 (l >> 4) + j][col0 + (l & 15)] from the K image (as lds_read_tr16)
template <int D>
PICO_DEV bf16x8 kimg_read_tr16(const char* base, int row0, int col0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int q = i >> 2, p = i & 3;
  const int col = col0 + 4 * p;
  const int chunk = col >> 3, sub = (col & 7) * 2;
  const int r0 = row0 + 8 * g + q;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + kimg_off<D>(r0, chunk) + sub));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + kimg_off<D>(r0 + 4, chunk) + sub));
  typedef __attribute__((ext_vector_type(8))) short i16x8;
  i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// delta[bh, q] = -sum_d dO * O (negated), lse2[bh, q] = LSE * log2(e); rows q in [Sq, Sq_pad) get
// delta = 0 and lse2 = +inf. Rows are ordered (b, h, q) so the LSE reads and the delta / lse2 writes are contiguous;
// each row of O / dO is one contiguous 2D-byte segment read by D/8 lanes.
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const pico_attn_args a, float* __restrict__ delta,
                                                           float* __restrict__ lse2, int sq_pad) {
  constexpr int LPR = D / 8;  // lanes per row (8 bf16 each)
  const int64_t rows = a.batch * a.heads_q * (int64_t)sq_pad;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  if (row >= rows) return;
  const int q = (int)(row % sq_pad);
  const int64_t bh = row / sq_pad;
  const int hq = (int)(bh % a.heads_q);
  const int b = (int)(bh / a.heads_q);
  if (q >= a.seqlen_q) {
    if (sub == 0) {
      delta[row] = 0.f;
      lse2[row] = INFINITY;
    }
    return;
  }
  const u16x8 ov = *reinterpret_cast<const u16x8*>((const bf16_t*)a.o + b * a.o_strides[0] + q * a.o_strides[1] +
                                                   hq * a.o_strides[2] + sub * 8);
  const u16x8 dv = *reinterpret_cast<const u16x8*>((const bf16_t*)a.dout + b * a.do_strides[0] +
                                                   q * a.do_strides[1] + hq * a.do_strides[2] + sub * 8);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += bf2f(ov[j]) * bf2f(dv[j]);
  // sum over the LPR (8 or 16) lanes of the row: DPP quad swaps + half-row mirror (+ row mirror)
  s += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0xB1, 0xF, 0xF, false));
  s += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x4E, 0xF, 0xF, false));
  s += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x141, 0xF, 0xF, false));
  if constexpr (LPR == 16) s += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x140, 0xF, 0xF, false));
  if (sub == 0) {
    delta[row] = -s;  // negated: it initialises the dP accumulator (dP - delta in the MFMA chain)
    lse2[row] = a.lse[bh * a.seqlen_q + q] * LOG2E;
  }
}

template <int D>
constexpr int bwd_waves_per_eu() { return D == 64 ? PICO_BWD_WAVES_PER_EU_D64 : 1; }

template <int D, bool CAUSAL>
__global__ __launch_bounds__(BwdCfg<D>::NTH, bwd_waves_per_eu<D>()) void attn_bwd_kernel(
    const pico_attn_args a, float scale, float scale_log2, const float* __restrict__ delta_g,
    const float* __restrict__ lse2_g, int sq_pad, float* __restrict__ dq_part, int64_t slab,
    float* __restrict__ trash, int hsplit, float* __restrict__ dkv_part, int kb0) {
  using C = BwdCfg<D>;
  constexpr int KS = C::KS, DT = C::DT, CPR = C::CPR, NW = C::NW;
  __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
  char* kimg = smem;
  char* ring = smem + C::KIMG;
  char* dsimg0 = smem + C::KIMG + C::NBUF * C::SLOT;  // dS^T [key][q] images: group u's tiles at (u % 2) G + j

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (scalar branches)
  const int r = lane & 31, h = lane >> 5;
  const int Sq = (int)a.seqlen_q, Sk = (int)a.seqlen_k;
#if PICO_BWD_STAMP
  __shared__ unsigned long long stamps[D == 64 ? 8 * STAMP_TILES * STAMP_PH : 1];  // D = 64 only (LDS)
  auto stamp = [&](int t, int ph) __attribute__((always_inline)) {
    const unsigned long long v = __builtin_amdgcn_s_memtime();
    if (D == 64 && lane == 0 && t < STAMP_TILES) stamps[(wave * STAMP_TILES + t) * STAMP_PH + ph] = v;
  };
#else
  auto stamp = [](int, int) __attribute__((always_inline)) {};
#endif
  const int Hq = (int)a.heads_q;
  const int G = (int)(a.heads_q / a.heads_kv);

  // heaviest key blocks first (causal: block 0 sees every query)
  // Small grids (GQA, few heads, short sequences): the (query head, query tile) list of a key block may
  // be split over `hsplit` workgroups (hs) so the grid fills the chip; each then writes fp32 dK/dV
  // partials that attn_bwd_dkv_kernel sums
  const int nbh = (int)(a.batch * a.heads_kv) * hsplit;
  const int kb = kb0 + (int)(blockIdx.x / nbh);  // key block; slab kb - kb0 of this launch
  const int bhs = blockIdx.x % nbh;
  const int hs = bhs % hsplit;
  const int bh = bhs / hsplit;
  const int b = bh / (int)a.heads_kv;
  const int hk = bh % (int)a.heads_kv;

  const int k0 = kb * BK;
  const int kw = k0 + 32 * wave;  // this wave's first key
  const int my_key = kw + r;

  const bf16_t* kg = (const bf16_t*)a.k + b * a.k_strides[0] + hk * a.k_strides[2];
  const bf16_t* vg = (const bf16_t*)a.v + b * a.v_strides[0] + hk * a.v_strides[2];

  const int qstart = CAUSAL ? k0 : 0;  // k0 is a multiple of BQ
  const int nqt = Sq > qstart ? (Sq - qstart + BQ - 1) / BQ : 0;
  const int ntot = G * nqt;  // tiles of this key block: (query head of the group, query tile)
  const int tb = (int)((int64_t)ntot * hs / hsplit);
  const int ntiles = (int)((int64_t)ntot * (hs + 1) / hsplit) - tb;
  const int hq0 = hk * G + tb / nqt, q00 = qstart + (tb % nqt) * BQ;  // first tile of this workgroup

  // ---- tile DMA: piece j is issued by wave j % NW ----
  //  j < NQP: Q rows RPP*j + lane / CPR, LDS chunk lane % CPR  <- source chunk (lane % CPR) ^ swz(row)
  //  j < 2 NQP: the same for dO;  j == 2 NQP: lanes 0-7 LSE*log2e[q0 .. q0+31], 8-15 delta (16..63 repeat)
  const int my_np = (C::NP / NW) + (wave < C::NP % NW ? 1 : 0);  // wave-uniform piece count
  int pc_row[C::NPW], pc_col[C::NPW], pc_kind[C::NPW];
  unsigned pc_dst[C::NPW];
#pragma unroll
  for (int i = 0; i < C::NPW; ++i) {
    const int j = wave + NW * i;
    if (j < 2 * C::NQP) {
      const int jj = j % C::NQP, row = C::RPP * jj + lane / CPR;
      pc_kind[i] = j < C::NQP ? 0 : 1;
      pc_row[i] = row;
      pc_col[i] = 8 * ((lane % CPR) ^ swz<D>(row));
      pc_dst[i] = (j < C::NQP ? 0 : C::QIMG) + jj * 1024;
    } else {
      const int l = lane & 15;
      pc_kind[i] = 2;
      pc_row[i] = 4 * (l & 7);
      pc_col[i] = l >> 3;  // 0: LSE, 1: delta
      pc_dst[i] = 2 * C::QIMG;
    }
  }
  // tile coordinates (query head, first query row), advanced incrementally (no per-tile divisions)
  struct Tc {
    int hq, q0;
  };
  const int qend = qstart + nqt * BQ;
  auto advance = [&](Tc& c) __attribute__((always_inline)) {
    c.q0 += BQ;
    if (c.q0 >= qend) {
      c.q0 = qstart;
      ++c.hq;
    }
  };
  auto next_slot = [](int si) __attribute__((always_inline)) { return si + 1 == C::NBUF ? 0 : si + 1; };
  const bf16_t* qbase = (const bf16_t*)a.q + b * a.q_strides[0];
  const bf16_t* dobase = (const bf16_t*)a.dout + b * a.do_strides[0];
  const unsigned delta_off = (unsigned)((const char*)delta_g - (const char*)lse2_g);  // same workspace
  const unsigned ring_lds = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr(smem)) + (unsigned)C::KIMG;
  auto issue = [&](int si, Tc c) __attribute__((always_inline)) {
    const int hq = c.hq, q0 = c.q0;
    const bool full = q0 + BQ <= Sq;
#pragma unroll
    for (int i = 0; i < C::NPW; ++i) {
      if (i < my_np) {
        const void* base;
        unsigned off;
        if (pc_kind[i] == 2) {  // lanes 0-7: LSE*log2e, 8-15: delta (pc_col), 4 rows each
          base = lse2_g + ((int64_t)b * Hq + hq) * sq_pad + q0;
          off = (unsigned)pc_row[i] * 4u + (pc_col[i] ? delta_off : 0u);
        } else {
          const int dq = full ? pc_row[i] : min(q0 + pc_row[i], Sq - 1) - q0;  // row within the tile
          if (pc_kind[i] == 0) {
            base = qbase + hq * a.q_strides[2] + (int64_t)q0 * a.q_strides[1];
            off = (unsigned)(dq * a.q_strides[1] + pc_col[i]) * 2u;
          } else {
            base = dobase + hq * a.do_strides[2] + (int64_t)q0 * a.do_strides[1];
            off = (unsigned)(dq * a.do_strides[1] + pc_col[i]) * 2u;
          }
        }
        dma_piece(base, off, ring_lds + (unsigned)si * (unsigned)C::SLOT + pc_dst[i]);
      }
    }
  };
  // the first PD tiles go out before the K/V prologue loads; nxt = coordinates of tile PD afterwards
  Tc nxt = {hq0, q00};
#pragma unroll
  for (int j = 0; j < C::PD; ++j) {
    if (j < ntiles) issue(j, nxt);
    advance(nxt);
  }

  // ---- K block -> LDS image; V fragments -> registers (B operand of dP = dO V^T) ----
  for (int id = threadIdx.x; id < BK * CPR; id += C::NTH) {
    const int row = id / CPR, ch = id % CPR;
    const int key = k0 + row;
    const u16x8 v = *reinterpret_cast<const u16x8*>(kg + (int64_t)min(key, Sk - 1) * a.k_strides[1] + ch * 8);
    *reinterpret_cast<u16x8*>(kimg + kimg_off<D>(row, ch)) = key < Sk ? v : (u16x8)0;
  }
  bf16x8 vf[KS];
  {
    const bool ok = my_key < Sk;
    const bf16_t* vp = vg + (int64_t)min(my_key, Sk - 1) * a.v_strides[1] + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(vp + 16 * ks);
      vf[ks] = __builtin_bit_cast(bf16x8, ok ? v : (u16x8)0);
    }
  }

  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    dk[dt] = (f32x16)0.f;
    dv[dt] = (f32x16)0.f;
  }

  auto slot_of = [&](int si) __attribute__((always_inline)) {
    return (const char*)(ring + (unsigned)si * (unsigned)C::SLOT);
  };
  // causal: a wave whose keys all lie past the tile's last query row has nothing to do for it
  auto active = [&](int q0) __attribute__((always_inline)) { return !CAUSAL || kw <= q0 + BQ - 1; };

  // S[q][key] and dP[q][key] of tile t: A = Q / dO rows (LDS), B = K^T (LDS) / V^T (registers)
  // Lane-constant LDS offsets of the per-tile operand reads (D = 64), computed once and pinned in
  // registers: an empty asm makes them opaque, so the compiler keeps 16 registers instead of
  // re-deriving the XOR swizzles (~100 VALU) every tile. Tile-dependent parts are slot bases and
  // immediate row deltas (16 Q/dO rows = 2 KiB: the swizzles depend on row bits 0-3 only).
  unsigned qo[KS], ko[KS], tro[DT][2], dso[4];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    qo[ks] = lds_off<D>(r, 2 * ks + h);
    ko[ks] = kimg_off<D>(32 * wave + r, 2 * ks + h);
  }
  {
    const int g = lane >> 4, i = lane & 15, hh = g >> 1, q = i >> 2, p = i & 3;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int col = 32 * dt + 16 * (g & 1) + 4 * p;
      tro[dt][0] = lds_off<D>(4 * hh + q, col >> 3) + (col & 7) * 2;
      tro[dt][1] = lds_off<D>(4 * hh + q + 8, col >> 3) + (col & 7) * 2;
    }
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) dso[g] = ds_img_off(32 * wave + r, 8 * g + 4 * h);
  if constexpr (D == 64) {
#pragma unroll
    for (int k = 0; k < KS; ++k) asm volatile("" : "+v"(qo[k]), "+v"(ko[k]));
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) asm volatile("" : "+v"(tro[dt][0]), "+v"(tro[dt][1]));
#pragma unroll
    for (int g = 0; g < 4; ++g) asm volatile("" : "+v"(dso[g]));
  }
  auto tr_pair = [](const char* base, unsigned lo_off, unsigned hi_off) __attribute__((always_inline)) {
    const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + lo_off));
    const i16x4 up = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + hi_off));
    typedef __attribute__((ext_vector_type(8))) short i16x8;
    i16x8 v = {lo[0], lo[1], lo[2], lo[3], up[0], up[1], up[2], up[3]};
    return __builtin_bit_cast(bf16x8, v);
  };

  // dP's accumulator starts at -delta of its rows (the tile's LSE/delta piece), so the chain yields
  // dP - delta directly
  auto sdp = [&](int si, f32x16& s, f32x16& dp) __attribute__((always_inline)) {
    const char* qs = slot_of(si);
    const char* dos = qs + C::QIMG;
    const float* nd = (const float*)(qs + 2 * C::QIMG) + 32;  // -delta[32]
    s = (f32x16)0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(nd + 8 * g + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) dp[4 * g + j] = v[j];
    }
    if constexpr (PICO_BWD_SCHED && D == 64) {  // D = 128: no registers for all 24 operands at once
      bf16x8 qa[KS], kbf[KS], da[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        qa[ks] = lds_read_b128(qs, qo[ks]);
        kbf[ks] = lds_read_b128(kimg, ko[ks]);
        da[ks] = lds_read_b128(dos, qo[ks]);
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s = mfma32(qa[ks], kbf[ks], s);
        dp = mfma32(da[ks], vf[ks], dp);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 3 * KS, 0);  // all operand reads first,
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * KS, 0);  // then the S / dP MFMAs
    } else {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 qa = lds_read_b128(qs, lds_off<D>(r, 2 * ks + h));
        const bf16x8 kbf = lds_read_b128(kimg, kimg_off<D>(32 * wave + r, 2 * ks + h));
        s = mfma32(qa, kbf, s);
        const bf16x8 da = lds_read_b128(dos, lds_off<D>(r, 2 * ks + h));
        dp = mfma32(da, vf[ks], dp);
      }
    }
  };

  // P = exp2(S * scale*log2e - LSE*log2e) (in s), dS = P * (dP - delta) (dp holds dP - delta); then
  // dV[key][d] += P^T dO, dK[key][d] += dS^T Q (k index = the tile's query rows). sf receives dS in
  // bf16 (the dK operand), reused for the dS^T image.
  auto softmax_dkdv = [&](int si, int q0, f32x16& s, const f32x16& dp, bf16x8 (&sf)[2]) __attribute__((always_inline)) {
    const char* qs = slot_of(si);
    const char* dos = qs + C::QIMG;
    const float* lsd = (const float*)(qs + 2 * C::QIMG);
    // rows of this lane's accumulator registers: q = 8g + 4h + (0..3), g = 0..3
    f32x4 l2[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) l2[g] = *reinterpret_cast<const f32x4*>(lsd + 8 * g + 4 * h);
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = fast_exp2(__builtin_fmaf(s[i], scale_log2, -l2[i >> 2][i & 3]));
    if ((CAUSAL && kw + 31 > q0) || (k0 + BK > Sk)) {  // wave-uniform
      // causal: key > q  <=>  (i&3) + 8(i>>2) < rel;  padding keys: key >= Sk
      const int rel = CAUSAL ? my_key - q0 - 4 * h : -1;
      const bool kill_all = my_key >= Sk;
#pragma unroll
      for (int i = 0; i < 16; ++i) s[i] = ((i & 3) + 8 * (i >> 2) < rel || kill_all) ? 0.f : s[i];
    }
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      float pv[8], sv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pv[j] = s[8 * st + j];
        sv[j] = s[8 * st + j] * dp[8 * st + j];
      }
      const bf16x8 pf = pack_frag(pv);
      sf[st] = pack_frag(sv);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const bf16x8 dof = D == 64 ? tr_pair(dos + 16 * st * C::RB, tro[dt][0], tro[dt][1])
                                   : lds_read_tr32<D>(dos, 16 * st, 32 * dt, lane);
        dv[dt] = mfma32(pf, dof, dv[dt]);
        const bf16x8 qf = D == 64 ? tr_pair(qs + 16 * st * C::RB, tro[dt][0], tro[dt][1])
                                  : lds_read_tr32<D>(qs, 16 * st, 32 * dt, lane);
        dk[dt] = mfma32(sf[st], qf, dk[dt]);
      }
    }
  };

  // dS^T image [key][q] (bf16) of tile t: elements 4g..4g+3 (sf[g / 2] half g % 2) are q = 8g + 4h + 0..3
  // -> one 8-B store each
  auto ds_write = [&](int par, const bf16x8 (&sf)[2]) __attribute__((always_inline)) {
    char* dsimg = dsimg0 + (unsigned)par * (unsigned)C::DSIMG;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      const bf16x8 v = sf[g >> 1];
      const bf16x4 w = (g & 1) ? bf16x4{v[4], v[5], v[6], v[7]} : bf16x4{v[0], v[1], v[2], v[3]};
      *reinterpret_cast<bf16x4*>(dsimg + dso[g]) = w;
    }
  };

  // dQ partial [q][d] = scale * dS[q][:] K[:][d] over this block's keys for tile t (16x16 tiles, one
  // (or two, D=128) per wave; both operands by transposed reads), stored fp32 into the key block's slab.
  // D = 64: the 16x16x32 key steps are software-pipelined, step i+1's four transposed reads issued
  // before step i's MFMA (reads of steps past kmax are harmless: in-bounds LDS, never consumed).
  auto dq_tile = [&](int par, Tc c) __attribute__((always_inline)) {
    const char* dsimg = dsimg0 + (unsigned)par * (unsigned)C::DSIMG;
    constexpr int NT = (BQ / 16) * (D / 16);
    int kmax = min(BK, Sk - k0);
    if (CAUSAL) kmax = min(kmax, c.q0 + BQ - k0);
    const int nst = (kmax + 31) >> 5;  // key steps (wave-uniform)
    const int g16 = lane >> 4, i16 = lane & 15;
    typedef __attribute__((ext_vector_type(8))) short i16x8;
#pragma unroll
    for (int tt = 0; tt < NT / NW; ++tt) {
      const int tl = wave + NW * tt;
      const int qi = tl / (D / 16), di = tl % (D / 16);
      const int qc = 16 * qi + 4 * (i16 & 3);
      // A = dS[q = 16 qi + (lane & 15)][key = kk + 8 g16 + j]: transposed read of the [key][q] image
      auto load = [&](int i, bf16x8& av, bf16x8& bv) __attribute__((always_inline)) {
        const int row = 32 * i + 8 * g16 + (i16 >> 2);
        const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(dsimg + ds_img_off(row, qc)));
        const i16x4 up = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(dsimg + ds_img_off(row + 4, qc)));
        const i16x8 v = {lo[0], lo[1], lo[2], lo[3], up[0], up[1], up[2], up[3]};
        av = __builtin_bit_cast(bf16x8, v);
        bv = kimg_read_tr16<D>(kimg, 32 * i, di * 16, lane);
      };
      f32x4 acc = (f32x4)0.f;
      if constexpr (D == 64) {
        bf16x8 a0, b0, a1, b1;
        load(0, a0, b0);
#pragma unroll
        for (int i = 0; i < BK / 32; i += 2) {
          load(i + 1, a1, b1);
          if (i < nst) acc = mfma16(a0, b0, acc);
          if (i + 2 < BK / 32) load(i + 2, a0, b0);
          if (i + 1 < nst) acc = mfma16(a1, b1, acc);
        }
      } else {  // D = 128: no registers for the second operand set
        for (int i = 0; i < nst; ++i) {
          bf16x8 a0, b0;
          load(i, a0, b0);
          acc = mfma16(a0, b0, acc);
        }
      }
      // every lane stores (rows past Sq go to a trash slot), so the per-tile count of vector-memory
      // instructions is fixed and the ring's vmcnt waits stay exact
      const int qr = c.q0 + qi * 16 + 4 * g16;  // this lane's first row
      float* dst = dq_part + (kb - kb0) * slab + ((int64_t)b * Sq + qr) * Hq * D + c.hq * D + di * 16 + i16;
      const int rs = Hq * D;  // row stride (elements)
      if (c.q0 + BQ <= Sq) {  // wave-uniform: whole tile in range
#pragma unroll
        for (int j = 0; j < 4; ++j) dst[j * rs] = acc[j] * scale;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) *(qr + j < Sq ? dst + j * rs : trash + lane) = acc[j] * scale;
      }
    }
  };

  // One barrier per group of G tiles: group u computes its tiles (S/dP -> P/dS -> dV/dK, dS images
  // (u % 2) G + j) and the dQ tiles of group u - 1, whose dS images the barrier published. The two
  // waves sharing a SIMD (w, w + 4) run them in opposite orders, so one's S/dP and dV/dK MFMAs overlap
  // the other's LDS-latency-bound dQ steps and softmax VALU instead of both waves contending for the
  // same unit in lockstep. The ring holds the tiles of groups u and u + 1 ... (PD = NBUF - G ahead):
  // group u issues the DMA of tiles uG + PD .. uG + PD + G - 1, whose slots held tiles of group u - 1
  // or earlier (retired before the barrier).
  // Per-wave vector-memory ops in issue order, group g: DMA pieces of its G look-ahead tiles, then the
  // dQ stores of group g - 1.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // K image and the prologue tiles visible
  constexpr int GT = C::G, PD = C::PD;  // tiles per barrier, look-ahead
  constexpr int NST = 4 * ((BQ / 16) * (D / 16) / NW);  // dQ stores per wave per tile
  auto tiles_in = [&](int lo, int hi) __attribute__((always_inline)) {  // |[lo, hi) ∩ [0, ntiles)|
    return max(0, min(hi, ntiles) - max(lo, 0));
  };
  const bool dq_first = PICO_BWD_STAGGER && D == 64 && wave >= NW / 2;  // D = 128: no registers to spare
  if constexpr (GT == 1) {  // one barrier per tile (D = 128: the variant below measured 3 % slower)
    Tc cur = {hq0, q00}, prev = cur;
    int si_cur = 0, si_nxt = PD;  // ring slots of tiles t and t + PD
    for (int t = 0; t < ntiles; ++t) {
      stamp(t, 0);
      // my pieces of tile t landed: issued in iteration j0 = t - PD, or in the prologue (j0 < 0)
      const int j0 = t - PD;
      if (j0 >= 0) {
        int younger = j0 >= 1 ? NST : 0;
        for (int j = j0 + 1; j < t; ++j) younger += (j + PD < ntiles ? my_np : 0) + (j >= 1 ? NST : 0);
        wait_vmcnt(younger);
      }
      // everyone's pieces of tile t visible, dS(t-1) visible, reads of slot (t-1) % NBUF and of
      // dS image t % 2 (dQ of t-2) retired
      lds_barrier();
      stamp(t, 1);
      if (t + PD < ntiles) issue(si_nxt, nxt);
      if (dq_first && t >= 1) dq_tile((t - 1) & 1, prev);
      stamp(t, 2);
      if (active(cur.q0)) {
        f32x16 s, dp;
        bf16x8 sf[2];
        sdp(si_cur, s, dp);
        softmax_dkdv(si_cur, cur.q0, s, dp, sf);
        stamp(t, 3);
        ds_write(t & 1, sf);
      }
      stamp(t, 4);
      if (!dq_first && t >= 1) dq_tile((t - 1) & 1, prev);
      stamp(t, 5);
      prev = cur;
      advance(cur);
      advance(nxt);
      si_cur = next_slot(si_cur);
      si_nxt = next_slot(si_nxt);
    }
    lds_barrier();
    if (ntiles > 0) dq_tile((ntiles - 1) & 1, prev);
  } else {
    Tc cur = {hq0, q00}, dqc = cur;  // tile t's coordinates; the next dQ tile's (G tiles behind)
    int si_cur = 0, si_nxt = PD;     // ring slots of tiles t and t + PD
    int pc = 0, pq = 0;              // dS images of tile t and of the next dQ tile ((tile) % 2G)
    auto next_img = [](int p) __attribute__((always_inline)) { return p + 1 == 2 * GT ? 0 : p + 1; };
    auto dq_next = [&]() __attribute__((always_inline)) {
      dq_tile(pq, dqc);
      advance(dqc);
      pq = next_img(pq);
    };
    int u = 0;
    for (int t0 = 0; t0 < ntiles; t0 += GT, ++u) {
      stamp(t0, 0);
      // my pieces of this group's tiles landed: the last one, tile tl, went out in group gi (or the
      // prologue); younger = the rest of gi's batch, gi's dQ stores, and every op of groups gi+1 .. u-1
      const int tl = min(t0 + GT, ntiles) - 1;
      if constexpr (PD == GT) {  // the group's pieces went out in group u - 1, before its G dQ tiles' stores
        if (u >= 1) wait_vmcnt(u >= 2 ? GT * NST : 0);
      } else if (tl - PD >= 0) {
        const int gi = (tl - PD) / GT;
        int younger = my_np * tiles_in(tl + 1, gi * GT + PD + GT) + (gi >= 1 ? GT * NST : 0);
        for (int g = gi + 1; g < u; ++g) younger += my_np * tiles_in(g * GT + PD, g * GT + PD + GT) + (g >= 1 ? GT * NST : 0);
        wait_vmcnt(younger);
      }
      // everyone's pieces of the group visible, the last group's dS images visible, reads of the slots
      // about to be refilled and of the dS images about to be rewritten (dQ of group u - 2) retired
      lds_barrier();
      stamp(t0, 1);
  #pragma unroll
      for (int j = 0; j < GT; ++j) {
        if (t0 + PD + j < ntiles) issue(si_nxt, nxt);
        advance(nxt);
        si_nxt = next_slot(si_nxt);
      }
  #pragma unroll PICO_BWD_GROUP_UNROLL
      for (int j = 0; j < GT; ++j) {
        if (dq_first && u >= 1) dq_next();
        stamp(t0 + j, 2);
        if (t0 + j < ntiles && active(cur.q0)) {
          f32x16 s, dp;
          bf16x8 sf[2];
          sdp(si_cur, s, dp);
          softmax_dkdv(si_cur, cur.q0, s, dp, sf);
          stamp(t0 + j, 3);
          ds_write(pc, sf);
        }
        stamp(t0 + j, 4);
        if (!dq_first && u >= 1) dq_next();
        stamp(t0 + j, 5);
        advance(cur);
        si_cur = next_slot(si_cur);
        pc = next_img(pc);
      }
    }
    lds_barrier();
    for (int t = (u - 1) * GT; t < ntiles; ++t) dq_next();  // the last group's dQ tiles
  }

#if PICO_BWD_STAMP
  if (D == 64 && blockIdx.x == 0) {
    unsigned long long* out = reinterpret_cast<unsigned long long*>(trash + 64);
    for (int i = lane; i < STAMP_TILES * STAMP_PH; i += 64)
      out[wave * STAMP_TILES * STAMP_PH + i] = stamps[wave * STAMP_TILES * STAMP_PH + i];
  }
#endif
  // ---- epilogue: dK = scale * acc, dV = acc; lane holds d = 32 dt + r, keys kw + acc_row(i, h) ----
  if (hsplit == 1) {
    bf16_t* dkg = (bf16_t*)a.dk + b * a.dk_strides[0] + hk * a.dk_strides[2];
    bf16_t* dvg = (bf16_t*)a.dv + b * a.dv_strides[0] + hk * a.dv_strides[2];
    // (PICO_ATTN_ROPE_BWD: dK is rotated back afterwards by the dQ-sum launch, which also covers
    // the dK rows — table gathers in this epilogue cost more than that pass)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kw + acc_row(i, h);
      if (key < Sk) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          dkg[(int64_t)key * a.dk_strides[1] + 32 * dt + r] = f2bf(dk[dt][i] * scale);
          dvg[(int64_t)key * a.dv_strides[1] + 32 * dt + r] = f2bf(dv[dt][i]);
        }
      }
    }
  } else {  // fp32 partials [hs][dK | dV][b][key][hk][D]
    const int64_t part = (int64_t)a.batch * Sk * a.heads_kv * D;
    float* pk = dkv_part + (int64_t)(2 * hs) * part + ((int64_t)b * Sk * a.heads_kv + hk) * D;
    float* pv = pk + part;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kw + acc_row(i, h);
      if (key < Sk) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          pk[(int64_t)key * a.heads_kv * D + 32 * dt + r] = dk[dt][i] * scale;
          pv[(int64_t)key * a.heads_kv * D + 32 * dt + r] = dv[dt][i];
        }
      }
    }
  }
}

// dq[b, q, h, :] = sum over key blocks kb (causal: kb * 256 <= q) of the fp32 partial slabs, summed in
// kb order (deterministic), optionally rotated back (PICO_ATTN_ROPE_BWD). A thread owns the 8-element
// pair of chunks d0 .. d0+7 and D/2 + d0 .. (so the rotation pairs are local). Writes bf16 (strided), or
// ADDS into an fp32 accumulator.
// rope_dk: the grid also covers the B * Sk * Hkv rows of dK (written un-rotated by attn_bwd_kernel's
// epilogue), rotated back in place.
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const pico_attn_args a, const float* __restrict__ dq_part,
                                                          int64_t slab, int nkb, int f32acc, int rope_dk, int kb0) {
  constexpr int TPR = D / 16;  // threads per row
  const int64_t rows = a.batch * a.seqlen_q * a.heads_q;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / TPR;
  const int d0 = (threadIdx.x % TPR) * 8;
  if (row >= rows) {
    const int64_t kr = row - rows;
    if (!rope_dk || kr >= a.batch * a.seqlen_k * a.heads_kv) return;
    const int hk = (int)(kr % a.heads_kv);
    const int64_t bk = kr / a.heads_kv;
    const int key = (int)(bk % a.seqlen_k);
    const int b = (int)(bk / a.seqlen_k);
    bf16_t* p = (bf16_t*)a.dk + b * a.dk_strides[0] + key * a.dk_strides[1] + hk * a.dk_strides[2] + d0;
    const u16x8 v1 = *reinterpret_cast<const u16x8*>(p), v2 = *reinterpret_cast<const u16x8*>(p + D / 2);
    float x1[8], x2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      x1[j] = bf2f(v1[j]);
      x2[j] = bf2f(v2[j]);
    }
    rope_bwd8(a, key, d0, x1, x2);
    u16x8 o1, o2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = f2bf(x1[j]);
      o2[j] = f2bf(x2[j]);
    }
    *reinterpret_cast<u16x8*>(p) = o1;
    *reinterpret_cast<u16x8*>(p + D / 2) = o2;
    return;
  }
  const int hq = (int)(row % a.heads_q);
  const int64_t bq = row / a.heads_q;
  const int q = (int)(bq % a.seqlen_q);
  const int b = (int)(bq / a.seqlen_q);
  const int last = CAUSAL ? min(nkb - 1, q / BK - kb0) : nkb - 1;  // slabs k = key blocks kb0 + k
  float x1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, x2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k <= last; ++k) {
    const f32x4* lo = reinterpret_cast<const f32x4*>(dq_part + k * slab + row * D + d0);
    const f32x4* hi = reinterpret_cast<const f32x4*>(dq_part + k * slab + row * D + D / 2 + d0);
    const f32x4 l0 = lo[0], l1 = lo[1], h0 = hi[0], h1 = hi[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x1[j] += l0[j];
      x1[4 + j] += l1[j];
      x2[j] += h0[j];
      x2[4 + j] += h1[j];
    }
  }
  if (a.flags & PICO_ATTN_ROPE_BWD) rope_bwd8(a, q, d0, x1, x2);
  if (f32acc) {
    float* dst = (float*)a.dq + b * a.dq_strides[0] + q * a.dq_strides[1] + hq * a.dq_strides[2] + d0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dst[j] += x1[j];
      dst[D / 2 + j] += x2[j];
    }
    return;
  }
  u16x8 o1, o2;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    o1[j] = f2bf(x1[j]);
    o2[j] = f2bf(x2[j]);
  }
  bf16_t* dst = (bf16_t*)a.dq + b * a.dq_strides[0] + q * a.dq_strides[1] + hq * a.dq_strides[2] + d0;
  *reinterpret_cast<u16x8*>(dst) = o1;
  *reinterpret_cast<u16x8*>(dst + D / 2) = o2;
}

// tile-list split of a key block (see attn_bwd_kernel): the smallest factor (<= 8) giving at least two
// workgroups per CU (512 = one launch wave of 256 CUs x 2), at most the block's query tile count
// Split key blocks until ONE launch (a group of at most PICO_BWD_KB_CAP key blocks) fills the chip once
// (one workgroup per CU: the kernel's LDS), twice under GQA, whose key blocks carry G query heads' tiles and
// need the finer split to balance (PICO_BWD_HSPLIT_GRID = 0: this rule). Filling it twice without GQA (the
// round-1 rule: 512 workgroups over all key blocks) doubled the fp32 dK/dV partials for no faster main kernel
// — Llama-2-7B/tp2 per rank (B 2, 16 heads, D 128, S 1024): causal 117.9 -> 105.9 us, non-causal 148.8 ->
// 117.3 us for the whole backward; GQA-4 at the same shape: 164.5 (8 parts) vs 167.8 (4 parts); counting every
// key block instead of one launch's would leave a grouped launch (S 4096) half the chip.
#ifndef PICO_BWD_KB_CAP
#define PICO_BWD_KB_CAP 8
#endif
#ifndef PICO_BWD_HSPLIT_GRID
#define PICO_BWD_HSPLIT_GRID 0
#endif
int hsplit_for(const pico_attn_args* a) {
  if (a->heads_kv <= 0 || a->heads_q % a->heads_kv != 0) return 1;  // rejected by the argument checks
  const int64_t nkb = (a->seqlen_k + BK - 1) / BK;
  const int64_t nblk = (nkb < PICO_BWD_KB_CAP ? nkb : PICO_BWD_KB_CAP) * a->batch * a->heads_kv;  // per launch
  const int64_t tiles = (a->heads_q / a->heads_kv) * ((a->seqlen_q + BQ - 1) / BQ);  // of key block 0
  if (nblk <= 0) return 1;
  const int64_t grid = PICO_BWD_HSPLIT_GRID > 0 ? PICO_BWD_HSPLIT_GRID
                                                : (int64_t)pico_num_cus() * (a->heads_q > a->heads_kv ? 2 : 1);
  int d = 1;
  while (d < 8 && nblk * d < grid && 2 * d <= tiles) d *= 2;
  return d;
}

int sq_padded(const pico_attn_args* a) { return (int)((a->seqlen_q + BQ - 1) / BQ) * BQ; }

// [lse2 | delta], each [B*Hq][Sq_pad] fp32, rounded up to 64 floats
int64_t lsd_floats(const pico_attn_args* a) {
  const int64_t n = a->batch * a->heads_q * (int64_t)sq_padded(a);
  return ((n + 63) / 64) * 64;
}

// Key blocks per launch of the fused kernel (PICO_BWD_KB_CAP, above): its dQ partial slabs (one fp32
// [B, Sq, Hq, D] per key block) are bounded by this many; longer sequences run the key blocks in groups, each
// group's slab sum added into an fp32 dQ (the slab workspace grew as S^2 / 256)
int kb_groups(const pico_attn_args* a) {
  const int64_t nkb = (a->seqlen_k + BK - 1) / BK;
  return (int)((nkb + PICO_BWD_KB_CAP - 1) / PICO_BWD_KB_CAP);
}

template <int D>
int launch_bwd(const pico_attn_args* a, hipStream_t s) {
  const int f32acc = (a->flags & PICO_ATTN_DQ_F32_ACCUM) != 0;
  const int sq_pad = sq_padded(a);
  const int nkb = (int)((a->seqlen_k + BK - 1) / BK);
  const int ngroups = kb_groups(a);
  const int kbcap = ngroups > 1 ? PICO_BWD_KB_CAP : nkb;  // slabs held at once
  float* lse2 = (float*)a->workspace;
  float* delta = lse2 + lsd_floats(a);
  float* dq_part = delta + lsd_floats(a);
  const int64_t slab = a->batch * a->seqlen_q * a->heads_q * D;
  float* trash = dq_part + (int64_t)kbcap * slab;
  // grouped: an fp32 dQ [B, Sq, Hq, D] after the slabs accumulates the groups (unless the caller's dQ is fp32)
  float* dq32 = (ngroups > 1 && !f32acc) ? trash + 64 + STAMP_BYTES / 4 : nullptr;
  const int64_t rows = a->batch * a->seqlen_q * a->heads_q;
  // attn_bwd_dq_kernel: D/16 threads per row; with ROPE_BWD on the one-workgroup-per-key-block grid it
  // also rotates the dK rows (the split grid's attn_bwd_dkv_kernel already did) — in the last group only
  const int rope_dk = (a->flags & PICO_ATTN_ROPE_BWD) && hsplit_for(a) == 1;
  const int64_t kv_rows = rope_dk ? a->batch * a->seqlen_k * a->heads_kv : 0;
  const int pre_blocks = pico_cdiv(a->batch * a->heads_q * (int64_t)sq_pad * (D / 8), 256);
  PICO_TRY(pico_launch(PICO_K_ATTN_BWD_PRE, "attn_bwd_pre", attn_bwd_pre_kernel<D>, dim3(pre_blocks), dim3(256), 0, s, *a, delta, lse2, sq_pad));
  const int hsplit = hsplit_for(a);
  // fp32 dK/dV partials (hsplit > 1) after the trash slot, the diagnostic stamps and dq32
  float* dkv_part = hsplit > 1 ? trash + 64 + STAMP_BYTES / 4 + (dq32 ? slab : 0) : nullptr;
  const float sl2 = a->softmax_scale * LOG2E;
  pico_attn_args ag = *a;  // the dQ-sum launches' view: grouped -> fp32 accumulate into dq32
  if (dq32) {
    if (hipMemsetAsync(dq32, 0, (size_t)slab * 4, s) != hipSuccess) return pico_set_error("pico_attn_bwd: memset failed");
    ag.dq = dq32;
    ag.dq_strides[0] = a->seqlen_q * a->heads_q * D;
    ag.dq_strides[1] = a->heads_q * D;
    ag.dq_strides[2] = D;
  }
  const int acc = (f32acc || dq32) ? 1 : 0;
  for (int g = 0; g < ngroups; ++g) {
    const int kb0 = g * kbcap, n = min(kbcap, nkb - kb0);
    const int64_t nblk = (int64_t)n * a->batch * a->heads_kv * hsplit;
    if (nblk > 0) {
      if (a->causal) {
        PICO_TRY(pico_launch(PICO_K_ATTN_BWD, "attn_bwd", attn_bwd_kernel<D, true>, dim3((int)nblk), dim3(BwdCfg<D>::NTH), 0, s, *a, a->softmax_scale, sl2, delta, lse2, sq_pad, dq_part, slab, trash, hsplit, dkv_part, kb0));
      } else {
        PICO_TRY(pico_launch(PICO_K_ATTN_BWD, "attn_bwd", attn_bwd_kernel<D, false>, dim3((int)nblk), dim3(BwdCfg<D>::NTH), 0, s, *a, a->softmax_scale, sl2, delta, lse2, sq_pad, dq_part, slab, trash, hsplit, dkv_part, kb0));
      }
    }
    const int rdk = (g == ngroups - 1) ? rope_dk : 0;
    const int row_blocks = pico_cdiv((rows + (rdk ? kv_rows : 0)) * (D / 16), 256);
    if (a->causal) {
      PICO_TRY(pico_launch(PICO_K_ATTN_BWD_DQ, "attn_bwd_dq", attn_bwd_dq_kernel<D, true>, dim3(row_blocks), dim3(256), 0, s, ag, dq_part, slab, n, acc, rdk, kb0));
    } else {
      PICO_TRY(pico_launch(PICO_K_ATTN_BWD_DQ, "attn_bwd_dq", attn_bwd_dq_kernel<D, false>, dim3(row_blocks), dim3(256), 0, s, ag, dq_part, slab, n, acc, rdk, kb0));
    }
  }
  if (hsplit > 1 && nkb > 0) {
    const int kv_blocks = pico_cdiv(a->batch * a->seqlen_k * a->heads_kv * (D / 16), 256);
    PICO_TRY(pico_launch(PICO_K_ATTN_BWD_DKV, "attn_bwd_dkv", attn_bwd_dkv_kernel<D>, dim3(kv_blocks), dim3(256), 0, s, *a, dkv_part, hsplit));
  }
  if (dq32) {  // dq32 (RoPE^-1 already applied per group: the rotation is linear) -> the caller's bf16 dQ
    pico_attn_args ac = *a;
    ac.flags = 0;
    const int row_blocks = pico_cdiv(rows * (D / 16), 256);
    PICO_TRY(pico_launch(PICO_K_ATTN_BWD_DQ, "attn_bwd_dq", attn_bwd_dq_kernel<D, false>, dim3(row_blocks), dim3(256), 0, s, ac, dq32, slab, 1, 0, 0, 0));
  }
  return 0;
}

}  // namespace

// Shared argument validation for forward and backward.
// split backward for head_dim 64 (attn_bwd_split.hip) and 128 (attn_bwd_split_d128.hip); PICO_BWD_SPLIT_D64=0 /
// PICO_BWD_SPLIT_D128=0 build the fused form with per-key-block dQ slabs instead
#ifndef PICO_BWD_SPLIT_D64
#define PICO_BWD_SPLIT_D64 1
#endif
#ifndef PICO_BWD_SPLIT_D128
#define PICO_BWD_SPLIT_D128 1
#endif
int64_t pico_attn_bwd_split_workspace(const pico_attn_args* a);
int pico_attn_bwd_split(const pico_attn_args* a, hipStream_t s);

int pico_attn_check_common(const pico_attn_args* a, const char* op) {
  PICO_REQUIRE(a, "%s: null args", op);
  PICO_REQUIRE(a->q && a->k && a->v, "%s: null q/k/v", op);
  PICO_REQUIRE(a->head_dim == 64 || a->head_dim == 128, "%s: head_dim=%lld unsupported (64 or 128)", op,
               (long long)a->head_dim);
  PICO_REQUIRE(a->batch >= 0 && a->seqlen_q >= 0 && a->seqlen_k >= 0 && a->heads_q >= 0 && a->heads_kv > 0,
               "%s: bad sizes", op);
  PICO_REQUIRE(a->heads_q % a->heads_kv == 0, "%s: heads_q=%lld not a multiple of heads_kv=%lld", op,
               (long long)a->heads_q, (long long)a->heads_kv);
  PICO_REQUIRE(!a->causal || a->seqlen_q == a->seqlen_k, "%s: causal requires seqlen_q == seqlen_k", op);
  PICO_REQUIRE(a->seqlen_q < (1 << 30) && a->seqlen_k < (1 << 30), "%s: sequence too long", op);
  const int64_t* st[3] = {a->q_strides, a->k_strides, a->v_strides};
  for (int i = 0; i < 3; ++i)
    for (int d = 0; d < 3; ++d) PICO_REQUIRE(st[i][d] % 8 == 0, "%s: strides must be multiples of 8 elements", op);
  PICO_REQUIRE(((uintptr_t)a->q | (uintptr_t)a->k | (uintptr_t)a->v) % 16 == 0, "%s: q/k/v must be 16-byte aligned",
               op);
  return 0;
}

extern "C" {

int64_t pico_attn_args_size(void) { return (int64_t)sizeof(pico_attn_args); }

int64_t pico_attn_bwd_workspace_bytes(const pico_attn_args* a) {
  if (PICO_BWD_SPLIT_D64 && a->head_dim == 64) return pico_attn_bwd_split_workspace(a);
  if (PICO_BWD_SPLIT_D128 && a->head_dim == 128) return pico_attn_bwd_split_workspace(a);
  // lse2, delta [B*Hq*Sq_pad] fp32 + one fp32 dQ partial slab [B, Sq, Hq, D] per 256-key block of a group
  // (at most PICO_BWD_KB_CAP; grouped: + an fp32 dQ accumulator unless the caller's dQ is fp32)
  const int64_t nkb = (a->seqlen_k + BK - 1) / BK;
  const int ng = kb_groups(a);
  const int64_t slab = a->batch * a->seqlen_q * a->heads_q * a->head_dim;
  const int64_t nslab = (ng > 1 ? PICO_BWD_KB_CAP : nkb) + ((ng > 1 && !(a->flags & PICO_ATTN_DQ_F32_ACCUM)) ? 1 : 0);
  // + 64 floats of trash for the dQ stores of padded query rows
  const int hs = hsplit_for(a);
  const int64_t dkv = hs > 1 ? 2 * hs * a->batch * a->seqlen_k * a->heads_kv * a->head_dim : 0;  // fp32 partials
  return (2 * lsd_floats(a) + nslab * slab + 64 + dkv) * 4 + STAMP_BYTES;
}

int pico_attn_bwd(const pico_attn_args* a, void* stream) {
  int rc = pico_attn_check_common(a, "pico_attn_bwd");
  if (rc) return rc;
  PICO_REQUIRE(a->o && a->lse && a->dout && a->dq && a->dk && a->dv && a->workspace, "pico_attn_bwd: null pointer");
  const int64_t* st[5] = {a->o_strides, a->do_strides, a->dq_strides, a->dk_strides, a->dv_strides};
  for (int i = 0; i < 5; ++i)
    for (int d = 0; d < 3; ++d)
      PICO_REQUIRE(st[i][d] % 8 == 0 || (i == 2 && (a->flags & PICO_ATTN_DQ_F32_ACCUM)),
                   "pico_attn_bwd: strides must be multiples of 8 elements");
  if (a->flags & PICO_ATTN_ROPE_BWD) {
    PICO_REQUIRE(!(a->flags & PICO_ATTN_DQ_F32_ACCUM), "pico_attn_bwd: ROPE_BWD cannot be combined with DQ_F32_ACCUM");
    PICO_REQUIRE(a->rope_cos && a->rope_sin && ((uintptr_t)a->rope_cos | (uintptr_t)a->rope_sin) % 16 == 0,
                 "pico_attn_bwd: ROPE_BWD needs 16-byte aligned cos/sin tables");
    PICO_REQUIRE(a->rope_stride % 8 == 0 && a->rope_stride >= a->head_dim / 2,
                 "pico_attn_bwd: bad rope table row stride %lld", (long long)a->rope_stride);
  }
  if (a->batch == 0 || a->seqlen_q == 0 || a->heads_q == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (a->head_dim == 64) return PICO_BWD_SPLIT_D64 ? pico_attn_bwd_split(a, s) : launch_bwd<64>(a, s);
  if (PICO_BWD_SPLIT_D128) return pico_attn_bwd_split(a, s);
  return launch_bwd<128>(a, s);
}

}  // extern "C"
