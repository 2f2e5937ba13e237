// Flash-attention backward for gfx950, split form (head_dim 64 here; 128 in attn_bwd_split_d128.hip): a query-major dQ kernel and a
// key-major dK/dV kernel instead of one kernel whose dQ needs a cross-workgroup reduction.
//
// Replaces flash-attn's backward of flash_attn_func (ref picotron/model.py:36) and the ring block
// backward ring_attention_backward (ref picotron/context_parallel/context_parallel.py:130-155):
//   P = exp(scale*QK^T - LSE), delta = rowsum(dO*O), dS = P*(dO V^T - delta),
//   dQ = scale * dS K, dK = scale * dS^T Q, dV = P^T dO.
//
// Why split: with one workgroup per key block, dQ is a sum over key blocks. At D = 64 that sum is one
// fp32 byte per 640 FLOPs — float atomics cap the kernel near a third of the MFMA peak and partial
// slabs cost O(S^2 / 256) workspace plus a read-back pass (VERDICT r01 "What's weak" 3).
// Here each output has exactly one owner and no reduction exists:
//   attn_bwd_q_kernel  (runs first): one workgroup = 4 waves = 128 query rows of one (batch, q-head),
//     sweeping 64-key tiles of K and V (LDS-DMA ring). Swapped products with the query on the lane:
//     S^T = K Q^T and dP^T = V dO^T (A = K / V rows from LDS, B = Q / dO fragments held in registers),
//     P^T and dS^T lane-local (LSE and delta are per-lane constants; dP starts from -delta as the
//     MFMA's C operand), dQ^T += K^T dS^T (A = transposed reads of the same K image, B = the dS^T
//     accumulator packed to bf16 in place). It also computes delta = rowsum(dO*O) from registers and
//     writes delta / LSE*log2(e) for the second kernel (no separate pre-pass).
//   attn_bwd_kv_kernel: one workgroup = 4 waves x 32 keys = 128 keys of one (batch, kv-head),
//     sweeping (query head of the group) x 32-row query tiles (Q, dO, LSE/delta by LDS-DMA). Key on
//     the lane: S = Q K^T, dP = dO V^T (K, V fragments resident in registers), then dV^T += dO^T P and
//     dK^T += Q^T dS with the P / dS accumulators as B operands (no LDS round trip at all).
// The dQ kernel recomputes S and dP (3 products per score there, 4 in the dK/dV kernel: 7 vs the fused
// form's 5), trading 40 % more MFMA work for no slabs, no atomics, no cross-wave dS exchange and no
// barrier other than the ring's.
// RoPE^-1 (PICO_ATTN_ROPE_BWD) is applied in both epilogues: the rotation pairs (d, d + D/2) sit in
// one lane (accumulator tiles dt and dt + D/64), so it is register-local.
#include "attn_common.h"

#include <algorithm>
#include <type_traits>



namespace {

constexpr int QB = 128;  // dq kernel: query rows per workgroup (4 waves x 32)
constexpr int KT = 64;   // dq kernel: keys per tile
// dkv kernel workgroup: 128 keys = 4 waves (one per SIMD) of 32 keys. Two or three workgroups resident per CU
// (kv_minb) overlap one's prologue (K/V fragments, first tiles) and epilogue (dK/dV stores) with the others' main
// loops, which the 8-wave 256-key form (one workgroup per CU) could not: C2 causal 62 vs 68 us. Measured and
// dropped: 64 keys per wave (69-71 vs 52 us), a tile-pipelined body carrying S / dP of tile
// t + 1 across the barrier (+6 % at D = 64, noise at D = 128), two tiles per barrier interval.
constexpr int KVB = 128;                  // dkv kernel: keys per workgroup
constexpr int KPW = 32, KH = KPW / 32, KNW = KVB / KPW;  // keys per wave (one 32-key half), waves per workgroup
constexpr int QT = 32;                    // dkv kernel: query rows per tile

// Diagnostic builds (scripts/gpu_attn_timeline.sh; results unchanged):
// PICO_BWDKV_WGSTAMP: diagnostic build — every dK/dV workgroup records s_memrealtime (100 MHz, chip-wide)
// at entry, loop start, loop end and after its stores drained (4 x 8 B per workgroup, grids <= 65536)
#ifndef PICO_BWDKV_WGSTAMP
#define PICO_BWDKV_WGSTAMP 0
#endif
// PICO_BWDQ_WGSTAMP: the same four stamps for every dQ workgroup (same workspace tail)
#ifndef PICO_BWDQ_WGSTAMP
#define PICO_BWDQ_WGSTAMP 0
#endif
// PICO_KVP_STAMP: diagnostic build — every wave of attn_bwd_kvp_kernel accumulates s_memtime (shader clock)
// deltas per phase of its tiles (wait, barrier, DMA issue, M1(A), M1(B), M2(A), M2(B)), the tile count, the block
// prologue / epilogue cycles and the wave's start / end clocks: 16 x 8 B per wave at
// stamp_out[(block * NW + wave) * 16] (NW = waves per workgroup; scripts/kvp_stamps.py)
#ifndef PICO_KVP_STAMP
#define PICO_KVP_STAMP 0
#endif
constexpr int64_t STAMP_BYTES = (PICO_BWDKV_WGSTAMP || PICO_BWDQ_WGSTAMP || PICO_KVP_STAMP) ? 65536 * 4 * 8 : 0;

// dQ kernel: ring slots and workgroups per CU the register budget is sized for. D = 64: 3 slots (48 KiB), three
// workgroups per CU at 168 VGPRs (the two 32-key halves of a tile in turn: C2 45.7 -> 44.1 us, S 4096 115.9 ->
// 107.4). D = 128: 2 slots (64 KiB), two workgroups per CU at 248 VGPRs (V's fragments read after the S chain):
// C4 dQ 36.5 -> 33.8 us, GQA-4 44.5 -> 39.4.
template <int D>
struct QCfg {
  static constexpr int KS = D / 16, DT = D / 32, CPR = D / 8, RB = 2 * D;
  static constexpr int MINB = D == 64 ? 3 : 2;   // workgroups per CU (register budget 168 / 248 VGPRs)
  static constexpr int IMG = KT * RB;            // one K (or V) tile image (lds_off<D> layout)
  static constexpr int SLOT = 2 * IMG;           // K | V
#ifndef PICO_Q_NBUF64
#define PICO_Q_NBUF64 3
#endif
  static constexpr int NBUF = D == 64 ? PICO_Q_NBUF64 : 2;   // ring slots; prefetch NBUF - 1
  static constexpr int RPP = 1024 / RB;        // image rows per 1-KiB DMA piece
  static constexpr int NP = SLOT / 1024;       // pieces per tile
  static constexpr int NPW = NP / 4;           // per wave
};

template <int D>
struct KVCfg {
  static constexpr int KS = D / 16, DT = D / 32, CPR = D / 8, RB = 2 * D;
  static constexpr int QIMG = QT * RB;   // one Q (or dO) tile image
  static constexpr int LSD = 1024;       // LSE*log2e [32] | -delta [32] (one DMA piece)
  static constexpr int SLOT = 2 * QIMG + LSD;
#ifndef PICO_KV_NBUF
#define PICO_KV_NBUF 3
#endif
  static constexpr int NBUF = PICO_KV_NBUF;  // ring slots
  static constexpr int PD = NBUF - 1;        // prefetch distance (tiles)
  static constexpr int RPP = 1024 / RB;
  static constexpr int NQP = QIMG / 1024;
  static constexpr int NP = 2 * NQP + 1;
  static constexpr int NPW = (NP + KNW - 1) / KNW;
};

// One-round causal schedule of the dK/dV kernel (round 5). A causal grid of one workgroup per 128-key block has
// blocks of unequal work (C2: 32, 28, ..., 4 query tiles per key block) and, at three workgroups per CU, 1024
// workgroups for 768 slots: the light blocks that do not fit the first round ran as a tail in a near-empty chip
// (blocks 6-7 from 39 to 52 us, one slot in three busy; profiles/r03_attn_wg_timelines.json). Grouped, each
// workgroup runs a short list of key blocks of one (batch, kv-head) one after the other, sized so that every
// head's groups fill exactly one round: with the CU's SIMD arbitration by age (the oldest of three resident
// workgroups runs a tile in ~1.15 us, the youngest in ~2.2), the groups dispatched first get the most work (host:
// block_groups). Same box, 3 interleaved rounds (profiles/r05_ab_attn_groups.jsonl): C2 dK/dV 57.4 -> 56.3 us,
// C4 (B 4, D 128, one workgroup per CU: 512 blocks -> 256 groups of equal work) 59.3 -> 58.4; the same grouping of
// the dQ kernel's query blocks measured slower (C2 42.8 -> 47.3 us, GQA-4 40.0 -> 43.9: its lightest-first front,
// q_front, frees slots early for the heavy blocks, which a one-round grid cannot), so the dQ grid stays plain.
// grp.n == 0: the plain grid, one block per workgroup.
constexpr int GRP_MAX = 16;  // groups per (batch, head)
struct BlkGroups {
  int n;                   // groups per (batch, head); 0 = one block per workgroup
  unsigned long long cnt;  // blocks in group g: nibble g (1..4)
  unsigned w[GRP_MAX];     // block ids of group g: byte j of w[g], j < its count (heaviest first)
};

// w[g] for a wave-uniform g without indexing the kernel-argument array (selects, no scratch copy)
PICO_DEV unsigned grp_sel(const BlkGroups& t, int g) {
  unsigned r = t.w[0];
#pragma unroll
  for (int i = 1; i < GRP_MAX; ++i) r = g == i ? t.w[i] : r;
  return r;
}

PICO_DEV float halves_sum2(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

PICO_DEV bf16x8 tr_pair(const char* base, unsigned lo_off, unsigned hi_off) {
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + lo_off));
  const i16x4 up = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + hi_off));
  typedef __attribute__((ext_vector_type(8))) short i16x8;
  i16x8 v = {lo[0], lo[1], lo[2], lo[3], up[0], up[1], up[2], up[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Per-lane byte offsets of the 32x32x16 transposed operand of a [rows][D] lds_off<D> image: rows
// 4 (lane >> 5) + ((lane & 15) >> 2) (+8 for the second read), columns 32 dt + 16 ((lane >> 4) & 1) +
// 4 (lane & 3). A read at row0 (a multiple of 16: the swizzles see row bits 0-3 only) adds row0 * 2D.
template <int D>
PICO_DEV void tr_offsets(int lane, unsigned (&tro)[D / 32][2]) {
  const int g = lane >> 4, i = lane & 15, hh = g >> 1, q = i >> 2, p = i & 3;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) {
    const int col = 32 * dt + 16 * (g & 1) + 4 * p;
    tro[dt][0] = lds_off<D>(4 * hh + q, col >> 3) + (col & 7) * 2;
    tro[dt][1] = lds_off<D>(4 * hh + q + 8, col >> 3) + (col & 7) * 2;
  }
}

// Accumulation into AGPR-resident accumulators (attn_bwd_kvp128_kernel: the VGPR-form build keeps every builtin MFMA's
// accumulator in VGPRs, which the wave cannot hold beside its S / dP pipeline; the same form in the D = 128 dQ
// kernel, two waves per SIMD, measured slower: C4 41.0 -> 44.8 us, profiles/r06_dq128_agpr/): the compiler sees an opaque
// instruction, so the asm carries what its hazard recognizer would add (s_nop 1: VALU write -> MFMA read of the
// packed operand, 2 wait states); the accumulators are AGPR-class from their zero-initialisation (no copies at the
// loop edge) and are read only after a drain (acc_drain: the last MFMA's write before any VALU read)
PICO_DEV void mfma32_acc(f32x16& acc, const bf16x8& x, const bf16x8& y) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(x), "v"(y));
}
PICO_DEV void acc_drain4(f32x16 (&v)[4]) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(v[0]), "+a"(v[1]), "+a"(v[2]), "+a"(v[3]));
}

// ------------------------------------------------------------------------------------------------
// dQ kernel (query-major)
// ------------------------------------------------------------------------------------------------
// (Round 5 measured and removed a pipelined form of this tile — the two 32-key halves as one hand-ordered stream
// of 24 MFMA slots at two workgroups per CU, as attn_bwd_kvp_kernel: C2 40.5 vs 40.6 us, profiles/r05_ab_kvp_qp.jsonl.)
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, QCfg<D>::MINB) void attn_bwd_q_kernel(const pico_attn_args a, float scale, float scale_log2,
                                                             float* __restrict__ lse2_g, float* __restrict__ delta_g,
                                                             int sq_pad, unsigned long long* __restrict__ stamp_out,
                                                             int nfront, float lse_mul, float lse_pad) {
  using C = QCfg<D>;
#if PICO_BWDQ_WGSTAMP
  unsigned long long wgs[4];
  wgs[0] = __builtin_amdgcn_s_memrealtime();
#endif
  constexpr int KS = C::KS, DT = C::DT, RB = C::RB;
  __shared__ __attribute__((aligned(16))) char smem[C::NBUF * C::SLOT];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int Sq = (int)a.seqlen_q, Sk = (int)a.seqlen_k;

  // causal dispatch order (a head's blocks sit nbh block ids apart): the `nfront` lightest query blocks
  // first, then the rest heaviest-first. nfront = the blocks a heaviest-first order leaves for after the
  // first round of resident workgroups: run there, in a near-empty chip, each paid its whole prologue
  // latency alone (C2: blocks 0-1 started at 27-29 us and ended at 36 of 40); run first (oldest, so
  // favoured by the SIMD arbitration) they finish early and hand their slots to the heavy blocks.
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
  const int64_t ksd = a.k_strides[1], vsd = a.v_strides[1];

  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + QB);
  const int ntiles = (kend + KT - 1) / KT;
  const int lim_last = CAUSAL ? min(qw + 31, Sk - 1) : Sk - 1;   // last key any row of the wave sees
  const int lim_first = CAUSAL ? min(qw, Sk - 1) : Sk - 1;       // keys <= this need no mask
  const int lim_lane = CAUSAL ? min(my_q, Sk - 1) : Sk - 1;      // this lane's row sees keys <= it

  // ---- DMA: piece j = wave + 4 i of a tile; j < NP/2: K image piece j, else V image piece j - NP/2 ----
  int src_row[C::NPW], src_col[C::NPW];
  unsigned dst_off[C::NPW];
  bool is_k[C::NPW];
#pragma unroll
  for (int i = 0; i < C::NPW; ++i) {
    const int j = wave + 4 * i;
    is_k[i] = j < C::NP / 2;
    const int jj = is_k[i] ? j : j - C::NP / 2;
    const int row = C::RPP * jj + lane / C::CPR;
    src_row[i] = row;
    src_col[i] = 8 * ((lane % C::CPR) ^ swz<D>(row));
    dst_off[i] = (is_k[i] ? 0u : (unsigned)C::IMG) + (unsigned)jj * 1024u;
  }
  const unsigned smem_lds = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr(smem));
  unsigned full_off[C::NPW];  // per-lane byte offsets within a full tile (computed once)
#pragma unroll
  for (int i = 0; i < C::NPW; ++i) full_off[i] = (unsigned)(src_row[i] * (is_k[i] ? ksd : vsd) + src_col[i]) * 2u;
  // K and V tile rows advance by constant byte strides: wave-uniform pointers, bumped per tile
  const int64_t kst = (int64_t)KT * ksd * 2, vst = (int64_t)KT * vsd * 2;
  const char* kp_nxt = (const char*)kg;
  const char* vp_nxt = (const char*)vg;
  auto issue_piece = [&](int tile, int slot_i, int i) __attribute__((always_inline)) {
    const unsigned slot = smem_lds + (unsigned)slot_i * (unsigned)C::SLOT;
    const int base = tile * KT;
    const int lastrow = Sk - 1 - base;  // rows past it are clamped (finite; masked by the softmax)
    const bool full = base + KT <= Sk;
    const char* tb = is_k[i] ? kp_nxt : vp_nxt;
    const unsigned off = full ? full_off[i]
                              : (unsigned)(min(src_row[i], lastrow) * (is_k[i] ? ksd : vsd) + src_col[i]) * 2u;
    dma_piece(tb, off, slot + dst_off[i]);
  };
  auto bump = [&]() __attribute__((always_inline)) {
    kp_nxt += kst;
    vp_nxt += vst;
  };
  auto issue = [&](int tile, int slot_i) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < C::NPW; ++i) issue_piece(tile, slot_i, i);
    bump();
  };
  constexpr int P = C::NBUF - 1;  // prefetch distance
#pragma unroll
  for (int t = 0; t < P; ++t)
    if (t < ntiles) issue(t, t);

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
  // consume the prologue loads here: otherwise the compiler's own vmcnt waits for them sit at their
  // first use inside the tile loop, where vmcnt also counts the ring's in-flight DMA (-> vmcnt(0) per tile)
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(qf[ks]), "+v"(df[ks]));
  const float dall = halves_sum2(dsum);
  const bool row_ok = my_q < Sq;
  const float delta = row_ok ? dall : 0.f;
  const float lse2 = row_ok ? a.lse[((int64_t)b * a.heads_q + hq) * Sq + my_q] * LOG2E : INFINITY;
  if (h == 0 && my_q < sq_pad) {  // for the dK/dV kernel (padding rows: P = 0, delta = 0)
    // attn_bwd_kv_kernel: LSE log2 e (+inf padding); attn_bwd_kvp_kernel: -LSE / scale (-inf padding)
    lse2_g[(int64_t)bh * sq_pad + my_q] = row_ok ? a.lse[((int64_t)b * a.heads_q + hq) * Sq + my_q] * lse_mul : lse_pad;
    delta_g[(int64_t)bh * sq_pad + my_q] = -delta;
  }

  // per-lane LDS offsets, pinned in registers (the compiler would otherwise re-derive the swizzles)
  unsigned ro[KS], tro[DT][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) ro[ks] = lds_off<D>(r, 2 * ks + h);
  tr_offsets<D>(lane, tro);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(ro[ks]));
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) asm volatile("" : "+v"(tro[dt][0]), "+v"(tro[dt][1]));

  f32x16 dq[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dq[dt] = (f32x16)0.f;
  const f32x16 ndelta = (f32x16)(-delta);
  const float nl2 = -lse2;

  // One 64-key tile: S^T, dP^T (8 + 8 MFMAs), P^T and dS^T in registers, dQ^T += K^T dS^T (8 MFMAs).
  // kb: the slot's K image (V image at +IMG). One body for every tile (the causal / padding mask is an
  // in-place branch on S), so the loop-carried dQ accumulators never move between registers.
  // the two 32-key halves of a tile one after the other (half the K / V fragments and S / dP registers
  // live at a time: room for a third workgroup per CU at D = 64)
  auto tile = [&](const char* kb, bool mask, int n0) __attribute__((always_inline)) {
    const char* vb = kb + C::IMG;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      // D = 128 at two workgroups per CU (248 VGPRs): V's fragments are read after the S chain has
      // consumed K's (32 fewer live VGPRs)
      constexpr bool seqv = D == 128;
      bf16x8 kf[KS], vf[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        kf[ks] = lds_read_b128(kb, ro[ks] + kt * 32 * RB);
        if (!seqv) vf[ks] = lds_read_b128(vb, ro[ks] + kt * 32 * RB);
      }
      f32x16 sc, dpc;
      if (mask) {
        const int rel = lim_lane - n0 - 4 * h;
        f32x16 m;
#pragma unroll
        for (int i = 0; i < 16; ++i) m[i] = (32 * kt + (i & 3) + 8 * (i >> 2)) <= rel ? 0.f : -INFINITY;
        sc = mfma32(kf[0], qf[0], m);
      } else {
        sc = mfma32(kf[0], qf[0], (f32x16)0.f);
      }
#pragma unroll
      for (int ks = 1; ks < KS; ++ks) sc = mfma32(kf[ks], qf[ks], sc);
      if constexpr (seqv) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) vf[ks] = lds_read_b128(vb, ro[ks] + kt * 32 * RB);
      }
      dpc = mfma32(vf[0], df[0], ndelta);
#pragma unroll
      for (int ks = 1; ks < KS; ++ks) dpc = mfma32(vf[ks], df[ks], dpc);
      float ds[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) ds[i] = fast_exp2(__builtin_fmaf(sc[i], scale_log2, nl2)) * dpc[i];
      const bf16x8 dsf[2] = {pack_bf16x8(ds), pack_bf16x8(ds + 8)};
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const char* rowb = kb + (32 * kt + 16 * st) * RB;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) dq[dt] = mfma32(tr_pair(rowb, tro[dt][0], tro[dt][1]), dsf[st], dq[dt]);
      }
    }
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // prologue tiles and loads landed
#if PICO_BWDQ_WGSTAMP
  wgs[1] = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
#endif
  // unrolled by the ring depth: every LDS read of a tile has a compile-time slot (immediate offsets)
  for (int t0 = 0; t0 < ntiles; t0 += C::NBUF) {
#pragma unroll
    for (int u = 0; u < C::NBUF; ++u) {
      const int t = t0 + u;
      if (t >= ntiles) break;
      if (t > 0) {  // tile t landed (this wave's pieces); the younger tiles stay in flight
        if constexpr (P == 2) {  // counts as immediates (a runtime wait_vmcnt(n) is a compare-and-branch chain)
          if (t + 1 < ntiles) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::NPW) : "memory");
          else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if constexpr (P == 1) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
          wait_vmcnt(min(P - 1, ntiles - 1 - t) * C::NPW);  // issued tiles after t stay in flight
        }
      }
      lds_barrier();  // every wave's pieces of tile t visible; slot (t + P) % NBUF no longer read
      const int n0 = t * KT;
      const bool busy = n0 <= lim_last;  // wave-uniform: some row of the wave sees some key of the tile
      if (t + P < ntiles) issue(t + P, (u + P) % C::NBUF);
      if (busy) tile(smem + u * C::SLOT, n0 + KT - 1 > lim_first, n0);
    }
  }

#if PICO_BWDQ_WGSTAMP
  wgs[2] = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
#endif
  // ---- epilogue: lane = query my_q, register i of tile dt = d 32 dt + acc_row(i, h) ----
  // (every lane stays: the bf16 store's lane exchange needs the whole wave; only row_ok lanes store)
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
    if (row_ok) {
      float* dst = (float*)a.dq + b * a.dq_strides[0] + hq * a.dq_strides[2] + (int64_t)my_q * a.dq_strides[1];
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float* p = dst + 32 * dt + 8 * g + 4 * h;
#pragma unroll
          for (int j = 0; j < 4; ++j) p[j] += dq[dt][4 * g + j] * scale;
        }
    }
  } else {
    bf16_t* dst = (bf16_t*)a.dq + b * a.dq_strides[0] + hq * a.dq_strides[2] + (int64_t)qc * a.dq_strides[1];
    store_row_bf16_x16<DT>(dst, h, row_ok, [&](int dt, int i) { return dq[dt][i] * scale; });
  }
#if PICO_BWDQ_WGSTAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  wgs[3] = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  if (wave == 0 && lane < 4 && blockIdx.x < 65536) stamp_out[blockIdx.x * 4 + lane] = wgs[lane & 3];
#endif
}

// ------------------------------------------------------------------------------------------------
// dK / dV kernel (key-major)
// ------------------------------------------------------------------------------------------------
template <int D, bool CAUSAL, int MINB>
__global__ __launch_bounds__(KNW * 64, MINB) void attn_bwd_kv_kernel(const pico_attn_args a, float scale, float scale_log2,
                                                              const float* __restrict__ lse2_g,
                                                              const float* __restrict__ delta_g, int sq_pad,
                                                              int hsplit, float* __restrict__ dkv_part,
                                                              unsigned long long* __restrict__ stamp_out,
                                                              const BlkGroups grp) {
  using C = KVCfg<D>;
  constexpr int KS = C::KS, DT = C::DT, CPR = C::CPR, RB = C::RB;
  __shared__ __attribute__((aligned(16))) char smem[C::NBUF * C::SLOT];

  const int lane0 = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int Sq = (int)a.seqlen_q, Sk = (int)a.seqlen_k;
  const int Hq = (int)a.heads_q;
  const int G = (int)(a.heads_q / a.heads_kv);
#if PICO_BWDKV_WGSTAMP
  unsigned long long wgs[4];
  wgs[0] = __builtin_amdgcn_s_memrealtime();
#endif

  // heaviest key blocks first (causal: block 0 sees every query; lightest-first fronts as in the dQ kernel
  // measured neutral here); small grids split a key block's (query head, query tile) list over `hsplit`
  // workgroups with fp32 partials (attn_bwd_dkv_kernel sums)
  const int nbh = (int)(a.batch * a.heads_kv) * hsplit;
  const int gi = blockIdx.x / nbh;  // the key block, or with a one-round schedule (grp.n > 0) the block group
  const int bhs = blockIdx.x % nbh;
  const int hs = bhs % hsplit;
  const int bh = bhs / hsplit;
  const int b = bh / (int)a.heads_kv, hk = bh % (int)a.heads_kv;
  // the group's key blocks one after the other (grp.n == 0: the one block gi)
  const unsigned gw = grp.n ? grp_sel(grp, gi) : 0u;
  const int nblk_wg = grp.n ? (int)((grp.cnt >> (4 * gi)) & 15ull) : 1;
#pragma clang loop unroll(disable)
  for (int jb = 0; jb < nblk_wg; ++jb) {
  const int kb = grp.n ? (int)((gw >> (8 * jb)) & 255u) : gi;
  if (jb > 0) lds_barrier();  // every wave is done with the ring before this block's prologue DMA refills it
  // the lane id through an opaque copy: nothing lane-dependent is hoisted out of the block loop and kept live
  // across the whole body (that cost 100-180 B of scratch per lane at these register budgets)
  int lane_l = lane0;
  asm volatile("" : "+v"(lane_l));
  const int lane = lane_l, r = lane & 31, h = lane >> 5;
  const int k0 = kb * KVB;
  const int kw = k0 + KPW * wave;  // this wave's first key

  const int qstart = CAUSAL ? k0 : 0;  // k0 is a multiple of QT
  const int nqt = Sq > qstart ? (Sq - qstart + QT - 1) / QT : 0;
  const int ntot = G * nqt;
  const int tb = (int)((int64_t)ntot * hs / hsplit);
  const int ntiles = (int)((int64_t)ntot * (hs + 1) / hsplit) - tb;
  const int hq0 = hk * G + (nqt ? tb / nqt : 0), q00 = qstart + (nqt ? tb % nqt : 0) * QT;

  // ---- tile DMA: piece j = wave + KNW i: Q pieces, dO pieces, then the LSE/delta piece ----
  int pc_row[C::NPW], pc_col[C::NPW], pc_kind[C::NPW];
  unsigned pc_dst[C::NPW];
#pragma unroll
  for (int i = 0; i < C::NPW; ++i) {
    const int j = wave + KNW * i;  // wave-uniform
    if (j < 2 * C::NQP) {
      const int jj = j % C::NQP, row = C::RPP * jj + lane / CPR;
      pc_kind[i] = j < C::NQP ? 0 : 1;
      pc_row[i] = row;
      pc_col[i] = 8 * ((lane % CPR) ^ swz<D>(row));
      pc_dst[i] = (j < C::NQP ? 0 : C::QIMG) + jj * 1024;
    } else {  // lanes 0-7: LSE*log2e rows 4l..4l+3; 8-15: -delta rows (16-63 repeat)
      const int l = lane & 15;
      pc_kind[i] = 2;
      pc_row[i] = 4 * (l & 7);
      pc_col[i] = l >> 3;
      pc_dst[i] = 2 * C::QIMG;
    }
  }
  // A tile = (query head hq, 32 query rows from q0). Each of this wave's pieces reads from one wave-uniform
  // source pointer (Q rows, dO rows or the lse2 row) advanced by a constant stride per tile: the per-tile
  // issue is one DMA instruction per piece (no 64-bit index arithmetic and no source select in the loop).
  const int64_t qs1 = a.q_strides[1] * 2, ds1 = a.do_strides[1] * 2;  // bytes per query row
  const char* const qbase = (const char*)((const bf16_t*)a.q + b * a.q_strides[0]);
  const char* const dobase = (const char*)((const bf16_t*)a.dout + b * a.do_strides[0]);
  int64_t pc_step[C::NPW];  // bytes per tile of piece i's source
#pragma unroll
  for (int i = 0; i < C::NPW; ++i) pc_step[i] = pc_kind[i] == 0 ? QT * qs1 : (pc_kind[i] == 1 ? QT * ds1 : QT * 4);
  struct Tc {
    int hq, q0;
    const char* p[C::NPW];
  };
  auto make_tc = [&](int hq, int q0) __attribute__((always_inline)) {
    Tc c;
    c.hq = hq;
    c.q0 = q0;
#pragma unroll
    for (int i = 0; i < C::NPW; ++i)
      c.p[i] = pc_kind[i] == 0 ? qbase + hq * a.q_strides[2] * 2 + q0 * qs1
             : pc_kind[i] == 1 ? dobase + hq * a.do_strides[2] * 2 + q0 * ds1
                               : (const char*)(lse2_g + ((int64_t)b * Hq + hq) * sq_pad + q0);
    return c;
  };
  const int qend = qstart + nqt * QT;
  auto advance = [&](Tc& c) __attribute__((always_inline)) {
    if (c.q0 + QT >= qend) {
      c = make_tc(c.hq + 1, qstart);
    } else {
      c.q0 += QT;
#pragma unroll
      for (int i = 0; i < C::NPW; ++i) c.p[i] += pc_step[i];
    }
  };
  const unsigned delta_off = (unsigned)((const char*)delta_g - (const char*)lse2_g);  // same workspace
  const unsigned ring_lds = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr(smem));
  // per-lane byte offsets of this wave's pieces within a full tile (computed once; partial tiles clamp)
  unsigned pc_off[C::NPW];
#pragma unroll
  for (int i = 0; i < C::NP / KNW; ++i) pc_off[i] = (unsigned)(pc_row[i] * (pc_kind[i] == 0 ? qs1 : ds1) + pc_col[i] * 2);
  const bool ragged = Sq % QT != 0;
  auto issue = [&](int si, const Tc& c) __attribute__((always_inline)) {
    const unsigned dst = ring_lds + (unsigned)si * (unsigned)C::SLOT;
#pragma unroll
    for (int i = 0; i < C::NPW; ++i) {
      if (i < C::NP / KNW) {
        unsigned off = pc_off[i];
        if (ragged && c.q0 + QT > Sq && pc_kind[i] != 2)  // partial tile: clamp rows past Sq - 1
          off = (unsigned)((min(c.q0 + pc_row[i], Sq - 1) - c.q0) * (pc_kind[i] == 0 ? qs1 : ds1) + pc_col[i] * 2);
        dma_piece(c.p[i], off, dst + pc_dst[i]);
      } else if (wave < C::NP % KNW) {
        // the tile's LSE / delta piece (wave 0 only, pc_kind 2): its per-lane offset is re-derived from the lane
        // id here instead of being held in a VGPR for the whole sweep — at 168 VGPRs that VGPR was spilled, and
        // its scratch reload's vmcnt(0) drained wave 0's whole DMA queue (two tiles of prefetch) every tile
        static_assert(C::NP % KNW == 1 && C::NP / KNW == C::NPW - 1, "the LSE / delta piece is wave 0's last");
        // (from an opaque copy of the lane id: a plain __lane_id() expression is loop-invariant and gets hoisted
        // out of the tile loop into that same long-lived, spilled VGPR)
        int l = lane0;
        asm volatile("" : "+v"(l));
        l &= 15;
        dma_piece(c.p[i], (unsigned)(16 * (l & 7)) + ((l >> 3) ? delta_off : 0u), dst + pc_dst[i]);
      }
    }
  };
  constexpr int PD = C::PD;
  Tc nxt = make_tc(hq0, q00);
#pragma unroll
  for (int j = 0; j < PD; ++j) {
    if (j < ntiles) issue(j, nxt);
    advance(nxt);
  }

  // ---- K, V fragments of this wave's 64 keys (B operands of S = Q K^T, dP = dO V^T) ----
  const bf16_t* kg = (const bf16_t*)a.k + b * a.k_strides[0] + hk * a.k_strides[2];
  const bf16_t* vg = (const bf16_t*)a.v + b * a.v_strides[0] + hk * a.v_strides[2];
  bf16x8 kf[KH][KS], vf[KH][KS];
#pragma unroll
  for (int kt = 0; kt < KH; ++kt) {
    const int key = kw + 32 * kt + r;
    const bool ok = key < Sk;
    const bf16_t* kp = kg + (int64_t)min(key, Sk - 1) * a.k_strides[1] + 8 * h;
    const bf16_t* vp = vg + (int64_t)min(key, Sk - 1) * a.v_strides[1] + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u16x8 kv = *reinterpret_cast<const u16x8*>(kp + 16 * ks);
      const u16x8 vv = *reinterpret_cast<const u16x8*>(vp + 16 * ks);
      kf[kt][ks] = __builtin_bit_cast(bf16x8, ok ? kv : (u16x8)0);
      vf[kt][ks] = __builtin_bit_cast(bf16x8, ok ? vv : (u16x8)0);
    }
  }

  // consume the loads before the loop (see attn_bwd_q_kernel)
#pragma unroll
  for (int kt = 0; kt < KH; ++kt)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(kf[kt][ks]), "+v"(vf[kt][ks]));

  f32x16 dk[DT][KH], dv[DT][KH];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int kt = 0; kt < KH; ++kt) {
      dk[dt][kt] = (f32x16)0.f;
      dv[dt][kt] = (f32x16)0.f;
    }

  unsigned qo[KS], tro[DT][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) qo[ks] = lds_off<D>(r, 2 * ks + h);
  tr_offsets<D>(lane, tro);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(qo[ks]));
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) asm volatile("" : "+v"(tro[dt][0]), "+v"(tro[dt][1]));

  const bool kpad = kw + KPW - 1 >= Sk;  // wave-uniform: some of the wave's keys are padding
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // prologue tiles visible
#if PICO_BWDKV_WGSTAMP
  wgs[1] = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
#endif

  // One 32-query tile = M1 (S = Q K^T and dP = dO V^T - delta: 8 MFMAs, mask and -delta in the C operand),
  // then V (P = exp2(S scale log2e - LSE log2e), dS = P dP: VALU) and M2 (dV^T += dO^T P, dK^T += Q^T dS:
  // 8 MFMAs with the packed accumulators as B operands). A tile wholly above the wave's keys (causal) is
  // masked to P = 0 rather than skipped (no per-wave branch around the body).
  auto m1 = [&](int si, int q0, f32x16 (&s)[KH], f32x16 (&dp)[KH]) __attribute__((always_inline)) {
    const char* qs = smem + (unsigned)si * (unsigned)C::SLOT;
    const char* dos = qs + C::QIMG;
    const float* lsd = (const float*)(qs + 2 * C::QIMG);
    bf16x8 qa[KS], da[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      qa[ks] = lds_read_b128(qs, qo[ks]);
    }
    f32x16 nd;  // rows of this lane's accumulator registers: q = q0 + 8 g + 4 h + (0..3)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(lsd + 32 + 8 * g + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) nd[4 * g + j] = v[j];
    }
    // The causal / padding mask enters as the C operand of each S chain's first MFMA (-inf where key > q or
    // key >= Sk, else 0): the branch covers only those MFMAs, the rest of the tile is straight-line code.
    if ((CAUSAL && kw + KPW - 1 > q0) || kpad) {  // wave-uniform: diagonal / wholly masked tiles, padding keys
#pragma unroll
      for (int kt = 0; kt < KH; ++kt) {
        const int key = kw + 32 * kt + r;
        // masked iff (i&3) + 8(i>>2) < rel: causal key > q, or every row for a padding key
        const int rel = key >= Sk ? 64 : (CAUSAL ? key - q0 - 4 * h : -1);
        f32x16 m;
#pragma unroll
        for (int i = 0; i < 16; ++i) m[i] = ((i & 3) + 8 * (i >> 2) < rel) ? -INFINITY : 0.f;
        s[kt] = mfma32(qa[0], kf[kt][0], m);
      }
    } else {
#pragma unroll
      for (int kt = 0; kt < KH; ++kt) s[kt] = mfma32(qa[0], kf[kt][0], (f32x16)0.f);
    }
    // the dO fragments are read once the S chain has consumed Q's (16 fewer live VGPRs: room for a third
    // workgroup per CU; C2 58.5 -> 56.1 us at two)
#pragma unroll
    for (int kt = 0; kt < KH; ++kt)
#pragma unroll
      for (int ks = 1; ks < KS; ++ks) s[kt] = mfma32(qa[ks], kf[kt][ks], s[kt]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) da[ks] = lds_read_b128(dos, qo[ks]);
#pragma unroll
    for (int kt = 0; kt < KH; ++kt) {
      dp[kt] = mfma32(da[0], vf[kt][0], nd);
#pragma unroll
      for (int ks = 1; ks < KS; ++ks) dp[kt] = mfma32(da[ks], vf[kt][ks], dp[kt]);
    }
  };
  // V: P = exp2(S scale log2e - LSE log2e), dS = P dP, packed to bf16 (the B operands of M2)
  auto read_l2 = [&](int si, f32x4 (&l2)[4]) __attribute__((always_inline)) {
    const float* lsd = (const float*)(smem + (unsigned)si * (unsigned)C::SLOT + 2 * C::QIMG);
#pragma unroll
    for (int g = 0; g < 4; ++g) l2[g] = *reinterpret_cast<const f32x4*>(lsd + 8 * g + 4 * h);
  };
  auto vsm_l2 = [&](const f32x4 (&l2)[4], const f32x16 (&s)[KH], const f32x16 (&dp)[KH], bf16x8 (&pf)[KH][2],
                    bf16x8 (&sf)[KH][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int kt = 0; kt < KH; ++kt) {
      float pv[16], sv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        pv[i] = fast_exp2(__builtin_fmaf(s[kt][i], scale_log2, -l2[i >> 2][i & 3]));
        sv[i] = pv[i] * dp[kt][i];
      }
      pf[kt][0] = pack_bf16x8(pv);
      pf[kt][1] = pack_bf16x8(pv + 8);
      sf[kt][0] = pack_bf16x8(sv);
      sf[kt][1] = pack_bf16x8(sv + 8);
    }
  };
  auto vsm = [&](int si, const f32x16 (&s)[KH], const f32x16 (&dp)[KH], bf16x8 (&pf)[KH][2], bf16x8 (&sf)[KH][2])
      __attribute__((always_inline)) {
    f32x4 l2[4];
    read_l2(si, l2);
    vsm_l2(l2, s, dp, pf, sf);
  };
  // M2: dV^T[d][key] += dO^T[d][q] P[q][key], dK^T[d][key] += Q^T[d][q] dS[q][key] (A = transposed reads)
  auto m2 = [&](int si, const bf16x8 (&pf)[KH][2], const bf16x8 (&sf)[KH][2]) __attribute__((always_inline)) {
    const char* qs = smem + (unsigned)si * (unsigned)C::SLOT;
    const char* dos = qs + C::QIMG;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const bf16x8 dot = tr_pair(dos + 16 * st * RB, tro[dt][0], tro[dt][1]);
        const bf16x8 qt = tr_pair(qs + 16 * st * RB, tro[dt][0], tro[dt][1]);
#pragma unroll
        for (int kt = 0; kt < KH; ++kt) {
          dv[dt][kt] = mfma32(dot, pf[kt][st], dv[dt][kt]);
          dk[dt][kt] = mfma32(qt, sf[kt][st], dk[dt][kt]);
        }
      }
  };

  // Unrolled by the ring depth: the slot of every LDS read is a compile-time constant (immediate offsets).
  // (Measured and dropped, C2 causal: a stagger of the two waves of each SIMD by one phase — +2 %; carrying
  // S / dP of tile t + 1 across the barrier so M1(t + 1) overlaps V(t) inside the wave — +6 %.)
  constexpr int NPMY_LO = C::NP / KNW;  // this wave's pieces per tile: NPMY_LO or NPMY_LO + 1
  int q0cur = q00;
  for (int t0 = 0; t0 < ntiles; t0 += C::NBUF) {
#pragma unroll
    for (int u = 0; u < C::NBUF; ++u) {
      const int t = t0 + u;
      if (t >= ntiles) break;
      if (t > 0) {
        // this wave's pieces of tile t landed; the next tile's may stay in flight
        if constexpr (C::PD == 2) {
          if (t + 2 <= ntiles) {  // this wave's pieces of tile t landed; the next tile's may stay in flight
            if (wave < C::NP % KNW) wait_vmcnt(NPMY_LO + 1);
            else wait_vmcnt(NPMY_LO);
          } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
        } else {
          const int younger = min(C::PD - 1, ntiles - 1 - t);  // issued tiles after t (still in flight)
          wait_vmcnt(younger * (wave < C::NP % KNW ? NPMY_LO + 1 : NPMY_LO));
        }
        lds_barrier();  // everyone's pieces visible; the slot of tile t - 1 is no longer read
      }
      if (t + PD < ntiles) issue((u + PD) % C::NBUF, nxt);
      advance(nxt);
      f32x16 s[KH], dp[KH];
      bf16x8 pf[KH][2], sf[KH][2];
      m1(u, q0cur, s, dp);
      if constexpr (D == 128) {
        // one wave per SIMD: nothing else hides the transposed reads' LDS latency, so all of M2's A operands
        // (2 x DT x 2 fragments, 64 VGPRs) are requested before the softmax VALU instead of just before their MFMAs
        // (C4 dK/dV 46.8-47.1 -> 45.3-45.4 us, S 4096 166-170 -> 161-164; profiles/r04_ab_kv_m2pre_d128.jsonl)
        const char* qs = smem + (unsigned)u * (unsigned)C::SLOT;
        const char* dos = qs + C::QIMG;
        f32x4 l2[4];
        read_l2(u, l2);
        bf16x8 od[2][DT], oq[2][DT];
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            od[st][dt] = tr_pair(dos + 16 * st * RB, tro[dt][0], tro[dt][1]);
            oq[st][dt] = tr_pair(qs + 16 * st * RB, tro[dt][0], tro[dt][1]);
          }
        __builtin_amdgcn_sched_barrier(0);
        vsm_l2(l2, s, dp, pf, sf);
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int dt = 0; dt < DT; ++dt)
#pragma unroll
            for (int kt = 0; kt < KH; ++kt) {
              dv[dt][kt] = mfma32(od[st][dt], pf[kt][st], dv[dt][kt]);
              dk[dt][kt] = mfma32(oq[st][dt], sf[kt][st], dk[dt][kt]);
            }
      } else {
        vsm(u, s, dp, pf, sf);
        m2(u, pf, sf);
      }
      q0cur = q0cur + QT >= qend ? qstart : q0cur + QT;
    }
  }

#if PICO_BWDKV_WGSTAMP
  wgs[2] = __builtin_amdgcn_s_memrealtime();
#endif
  // ---- epilogue: lane = key kw + 32 kt + r, register i of tile dt = d 32 dt + acc_row(i, h) ----
  if (hsplit == 1) {
    const bool rope = (a.flags & PICO_ATTN_ROPE_BWD) != 0;
#pragma unroll
    for (int kt = 0; kt < KH; ++kt) {
      const int key = kw + 32 * kt + r;
      const int kc = min(key, Sk - 1);  // every lane runs the stores' lane exchange; only key < Sk store
      if (rope) {
        const bf16_t* cp = (const bf16_t*)a.rope_cos + (int64_t)kc * a.rope_stride;
        const bf16_t* sp = (const bf16_t*)a.rope_sin + (int64_t)kc * a.rope_stride;
#pragma unroll
        for (int dt = 0; dt < DT / 2; ++dt)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const u16x4 c4 = *reinterpret_cast<const u16x4*>(cp + 32 * dt + 8 * g + 4 * h);
            const u16x4 s4 = *reinterpret_cast<const u16x4*>(sp + 32 * dt + 8 * g + 4 * h);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float cf = bf2f(c4[j]), sn = bf2f(s4[j]);
              const float x1 = dk[dt][kt][4 * g + j], x2 = dk[dt + DT / 2][kt][4 * g + j];
              dk[dt][kt][4 * g + j] = x1 * cf + x2 * sn;
              dk[dt + DT / 2][kt][4 * g + j] = x2 * cf - x1 * sn;
            }
          }
      }
      bf16_t* dkp = (bf16_t*)a.dk + b * a.dk_strides[0] + hk * a.dk_strides[2] + (int64_t)kc * a.dk_strides[1];
      bf16_t* dvp = (bf16_t*)a.dv + b * a.dv_strides[0] + hk * a.dv_strides[2] + (int64_t)kc * a.dv_strides[1];
      store_row_bf16_x16<DT>(dkp, h, key < Sk, [&](int dt, int i) { return dk[dt][kt][i] * scale; });
      store_row_bf16_x16<DT>(dvp, h, key < Sk, [&](int dt, int i) { return dv[dt][kt][i]; });
    }
  } else {  // fp32 partials [hs][dK | dV][b][key][hk][D]
    const int64_t part = a.batch * a.seqlen_k * a.heads_kv * D;
    float* pk = dkv_part + (int64_t)(2 * hs) * part + ((int64_t)b * Sk * a.heads_kv + hk) * D;
    float* pv = pk + part;
#pragma unroll
    for (int kt = 0; kt < KH; ++kt) {
      const int key = kw + 32 * kt + r;
      if (key >= Sk) continue;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 wk, wv;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            wk[j] = dk[dt][kt][4 * g + j] * scale;
            wv[j] = dv[dt][kt][4 * g + j];
          }
          const int64_t o = (int64_t)key * a.heads_kv * D + 32 * dt + 8 * g + 4 * h;
          *reinterpret_cast<f32x4*>(pk + o) = wk;
          *reinterpret_cast<f32x4*>(pv + o) = wv;
        }
    }
  }
  }  // key blocks of the group
#if PICO_BWDKV_WGSTAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  wgs[3] = __builtin_amdgcn_s_memrealtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);
  if (wave == 0 && lane < 4 && blockIdx.x < 65536) stamp_out[blockIdx.x * 4 + lane] = wgs[lane & 3];
#endif
}

#ifndef PICO_SPLIT_D128_TU
// ------------------------------------------------------------------------------------------------
// dK / dV kernel, D = 64, 64-row query tiles in a hand-ordered stream (round 5; the default up to 1536 causal /
// 4096 non-causal keys, kvp_enabled)
// ------------------------------------------------------------------------------------------------
// The same work as attn_bwd_kv_kernel (key on the lane, 32 keys per wave, NW = 4 or 8 waves = 128 or 256 keys per
// workgroup, K / V fragments resident), but each ring tile is 64 query rows, two 32-row halves A and B whose phases interleave inside one
// wave: M1 = S and dP (8 MFMAs per half), V = the softmax VALU (P = exp2(c S'), dS = P dP, packed to bf16), M2 =
// dV^T += dO^T P and dK^T += Q^T dS (8 MFMAs per half). The 32-row kernel's tile is one dependency chain
// (M1 -> V -> M2, every operand read right before its MFMA: 19 waits per tile, ~1 us per tile for a wave
// alone); here a tile is the stream
//     M1(A) | reads of B's operands,  M1(B) | V(A) + A's transposed reads,  M2(A) | V(B) + B's reads,  M2(B)
// so every MFMA gap carries independent work (the guide's per-gap budget: <= 5 fillers, one transcendental),
// one barrier and one DMA round serve 64 rows, and two waves per SIMD (two 4-wave or one 8-wave workgroup per CU,
// <= 256 VGPRs) fill each other's remaining gaps. Row constants enter as the initial accumulators (no subtraction, no LSE
// registers): S' = Q K^T - LSE / scale (the dQ kernel writes -LSE / scale for these rows, -inf for padding
// rows; the causal / padding-key mask sets -inf in that initial value on diagonal tiles) and dP' = dO V^T - delta.
constexpr int QT2 = 64;
struct KVPCfg {
  static constexpr int D = 64, KS = 4, DT = 2, CPR = 8, RB = 128;
  static constexpr int QIMG = QT2 * RB;          // one Q (or dO) 64-row image, 8 KiB
  static constexpr int LSD = 1024;               // -LSE/scale [64] | -delta [64] (+ 512 B the DMA piece repeats)
  static constexpr int SLOT = 2 * QIMG + LSD;    // 17 KiB; 3 slots = 51 KiB per workgroup
#ifndef PICO_KVP_NBUF
#define PICO_KVP_NBUF 3
#endif
  static constexpr int NBUF = PICO_KVP_NBUF, PD = NBUF - 1;  // ring slots, prefetch distance (tiles)
  static constexpr int RPP = 1024 / RB;          // 8 image rows per 1-KiB piece
  static constexpr int NQP = QIMG / 1024;        // 8 pieces per image
  static constexpr int NP = 2 * NQP + 1;         // 17 pieces per tile: 4 per wave + wave 0's LSE / delta piece
};

#define KVP_SLOT() __builtin_amdgcn_sched_barrier(0)

template <bool CAUSAL, int MINB, int NW>
__global__ __launch_bounds__(NW * 64, MINB) void attn_bwd_kvp_kernel(const pico_attn_args a, float scale, float c2,
                                                                const float* __restrict__ sinit_g,
                                                                const float* __restrict__ delta_g, int sq_pad,
                                                                int hsplit, float* __restrict__ dkv_part,
                                                                const BlkGroups grp,
                                                                unsigned long long* __restrict__ stamp_out) {
  using C = KVPCfg;
#if PICO_KVP_STAMP
  unsigned long long ph[16] = {0}, tlast = 0, tblk = 0;
  ph[10] = __builtin_amdgcn_s_memrealtime();
  ph[12] = __builtin_amdgcn_s_memtime();
#define KVP_ST(i)                                          \
  {                                                        \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    ph[i] += t_ - tlast;                                   \
    tlast = t_;                                            \
  }
#else
#define KVP_ST(i)
#endif
  constexpr int KS = C::KS, DT = C::DT, CPR = C::CPR, RB = C::RB;
  // NW waves x 32 keys per block; each wave issues PPW of a tile's 16 image pieces (the first half Q, the second
  // dO), wave 0 also the LSE / delta piece
  constexpr int PPW = 2 * C::NQP / NW, KB = 32 * NW;
  static_assert(C::NP == PPW * NW + 1 && (PPW == 2 || PPW == 4), "Q / dO pieces per wave + one LSE / delta piece");
  __shared__ __attribute__((aligned(16))) char smem[C::NBUF * C::SLOT];

  const int lane0 = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int Sq = (int)a.seqlen_q, Sk = (int)a.seqlen_k;
  const int Hq = (int)a.heads_q;
  const int G = (int)(a.heads_q / a.heads_kv);
  const int nbh = (int)(a.batch * a.heads_kv) * hsplit;
  const int gi = blockIdx.x / nbh;
  const int bhs = blockIdx.x % nbh;
  const int hs = bhs % hsplit;
  const int bh = bhs / hsplit;
  const int b = bh / (int)a.heads_kv, hk = bh % (int)a.heads_kv;
  const unsigned gw = grp.n ? grp_sel(grp, gi) : 0u;
  const int nblk_wg = grp.n ? (int)((grp.cnt >> (4 * gi)) & 15ull) : 1;
  const unsigned delta_off = (unsigned)((const char*)delta_g - (const char*)sinit_g);  // same workspace
  const unsigned ring_lds = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr(smem));
#pragma clang loop unroll(disable)
  for (int jb = 0; jb < nblk_wg; ++jb) {
#if PICO_KVP_STAMP
  tblk = __builtin_amdgcn_s_memtime();
#endif
  const int kb = grp.n ? (int)((gw >> (8 * jb)) & 255u) : gi;
  if (jb > 0) lds_barrier();
  int lane_l = lane0;
  asm volatile("" : "+v"(lane_l));
  const int lane = lane_l, r = lane & 31, h = lane >> 5;
  const int k0 = kb * KB;
  const int kw = k0 + 32 * wave;
  const int qstart = CAUSAL ? k0 : 0;  // k0 is a multiple of QT2
  const int nqt = Sq > qstart ? (Sq - qstart + QT2 - 1) / QT2 : 0;
  const int ntot = G * nqt;
  const int tb = (int)((int64_t)ntot * hs / hsplit);
  const int ntiles = (int)((int64_t)ntot * (hs + 1) / hsplit) - tb;
  const int hq0 = hk * G + (nqt ? tb / nqt : 0), q00 = qstart + (nqt ? tb % nqt : 0) * QT2;

  // ---- tile DMA: this wave's pieces i = 0..3 are image pieces j = wave + 4 i (Q: j < 8, dO: 8 <= j < 16);
  // wave 0 also issues the LSE / delta piece (lanes 0-15: -LSE/scale rows 4l..4l+3, 16-31: -delta rows, 32-63
  // repeat 0-31)
  const int64_t qs1 = a.q_strides[1] * 2, ds1 = a.do_strides[1] * 2;  // bytes per query row
  const char* const qbase = (const char*)((const bf16_t*)a.q + b * a.q_strides[0]);
  const char* const dobase = (const char*)((const bf16_t*)a.dout + b * a.do_strides[0]);
  int pc_row[PPW];
  unsigned pc_off[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int jj = (wave + NW * i) % C::NQP;
    pc_row[i] = C::RPP * jj + lane / CPR;
    pc_off[i] = (unsigned)(pc_row[i] * (i < PPW / 2 ? qs1 : ds1) + 8 * ((lane % CPR) ^ swz<64>(pc_row[i])) * 2);
  }
  struct Tc {
    int hq, q0;
    const char* qp;
    const char* dp;
    const char* lp;
  };
  auto make_tc = [&](int hq, int q0) __attribute__((always_inline)) {
    Tc c;
    c.hq = hq;
    c.q0 = q0;
    c.qp = qbase + hq * a.q_strides[2] * 2 + q0 * qs1;
    c.dp = dobase + hq * a.do_strides[2] * 2 + q0 * ds1;
    c.lp = (const char*)(sinit_g + ((int64_t)b * Hq + hq) * sq_pad + q0);
    return c;
  };
  const int qend = qstart + nqt * QT2;
  auto advance = [&](Tc& c) __attribute__((always_inline)) {
    if (c.q0 + QT2 >= qend) {
      c = make_tc(c.hq + 1, qstart);
    } else {
      c.q0 += QT2;
      c.qp += QT2 * qs1;
      c.dp += QT2 * ds1;
      c.lp += QT2 * 4;
    }
  };
  const bool ragged = Sq % QT2 != 0;
  // one of this wave's pieces of a tile: i < PPW the image pieces, i == PPW the LSE / delta piece (wave 0 only)
  auto issue_piece = [&](int si, const Tc& c, int i) __attribute__((always_inline)) {
    const unsigned dst = ring_lds + (unsigned)si * (unsigned)C::SLOT;
    if (i < PPW) {
      const int jj = (wave + NW * i) % C::NQP;
      unsigned off = pc_off[i];
      if (ragged && c.q0 + QT2 > Sq) {  // partial tile: rows past Sq - 1 clamped (finite; their LSE is +inf)
        int l2 = lane0;
        asm volatile("" : "+v"(l2));
        const int row = C::RPP * jj + (l2 & 63) / CPR;
        off = (unsigned)((min(c.q0 + row, Sq - 1) - c.q0) * (i < PPW / 2 ? qs1 : ds1) +
                         8 * (((l2 & 63) % CPR) ^ swz<64>(row)) * 2);
      }
      dma_piece(i < PPW / 2 ? c.qp : c.dp, off, dst + (i < PPW / 2 ? 0u : (unsigned)C::QIMG) + (unsigned)jj * 1024u);
    } else if (wave == 0) {
      int l = lane0;
      asm volatile("" : "+v"(l));
      l &= 31;
      dma_piece(c.lp, (unsigned)(16 * (l & 15)) + ((l >> 4) ? delta_off : 0u), dst + 2u * C::QIMG);
    }
  };
  auto issue = [&](int si, const Tc& c) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i <= PPW; ++i) issue_piece(si, c, i);
  };
  Tc nxt = make_tc(hq0, q00);
#pragma unroll
  for (int j = 0; j < C::PD; ++j) {
    if (j < ntiles) issue(j, nxt);
    advance(nxt);
  }

  // ---- K, V fragments of this wave's 32 keys (B operands of S and dP) ----
  const bf16_t* kg = (const bf16_t*)a.k + b * a.k_strides[0] + hk * a.k_strides[2];
  const bf16_t* vg = (const bf16_t*)a.v + b * a.v_strides[0] + hk * a.v_strides[2];
  bf16x8 kf[KS], vf[KS];
  {
    const int key = kw + r;
    const bool ok = key < Sk;
    const bf16_t* kp = kg + (int64_t)min(key, Sk - 1) * a.k_strides[1] + 8 * h;
    const bf16_t* vp = vg + (int64_t)min(key, Sk - 1) * a.v_strides[1] + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u16x8 kv = *reinterpret_cast<const u16x8*>(kp + 16 * ks);
      const u16x8 vv = *reinterpret_cast<const u16x8*>(vp + 16 * ks);
      kf[ks] = __builtin_bit_cast(bf16x8, ok ? kv : (u16x8)0);
      vf[ks] = __builtin_bit_cast(bf16x8, ok ? vv : (u16x8)0);
    }
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(kf[ks]), "+v"(vf[ks]));
  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    dk[dt] = (f32x16)0.f;
    dv[dt] = (f32x16)0.f;
  }
  unsigned qo[KS], tro[DT][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) qo[ks] = lds_off<64>(r, 2 * ks + h);
  tr_offsets<64>(lane, tro);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(qo[ks]));
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) asm volatile("" : "+v"(tro[dt][0]), "+v"(tro[dt][1]));
  const bool kpad = kw + 31 >= Sk;  // wave-uniform: some of the wave's keys are padding
  const int mykey = kw + r;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // the initial accumulator of half X (rows 32 X + 8 g + 4 h + j of the lane's registers 4 g + j) from the
  // tile's LSE / delta piece: which = 0 -> -LSE/scale, 1 -> -delta
  auto init_rows = [&](const float* lsd, int X, int which) __attribute__((always_inline)) {
    f32x16 v;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 t4 = *reinterpret_cast<const f32x4*>(lsd + 64 * which + 32 * X + 8 * g + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[4 * g + j] = t4[j];
    }
    return v;
  };
  // diagonal / padding-key mask on an S initial value: -inf where key > query row (causal) or key >= Sk
  auto mask_rows = [&](f32x16& s, int qrow0) __attribute__((always_inline)) {
    const int rel = mykey >= Sk ? 1 << 30 : (CAUSAL ? mykey - qrow0 - 4 * h : -1);
#pragma unroll
    for (int i = 0; i < 16; ++i) s[i] = ((i & 3) + 8 * (i >> 2) < rel) ? -INFINITY : s[i];
  };
#if PICO_KVP_STAMP
  ph[8] += __builtin_amdgcn_s_memtime() - tblk;  // prologue of this block
#endif
  int q0cur = q00;
  for (int t0 = 0; t0 < ntiles; t0 += C::NBUF) {
#pragma unroll
    for (int u = 0; u < C::NBUF; ++u) {
      const int t = t0 + u;
      if (t >= ntiles) break;
#if PICO_KVP_STAMP
      tlast = __builtin_amdgcn_s_memtime();
      ph[7] += 1;
#endif
      if (t > 0) {
        // this wave's pieces of tile t landed; those of the younger tiles already issued stay in flight (counts as
        // immediates: a runtime wait_vmcnt(n) compiles to a compare-and-branch chain, ~12 branches per tile)
        if constexpr (C::PD == 2) {
          if (t + 1 < ntiles) {
            if (wave == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW + 1) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
          } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
        } else {
          const int younger = min(C::PD - 1, ntiles - 1 - t);
          wait_vmcnt(younger * (wave == 0 ? PPW + 1 : PPW));
        }
        KVP_ST(0);
        lds_barrier();  // every wave's pieces of tile t visible; the slot of tile t - 1 is no longer read
        KVP_ST(1);
      }
      // the DMA of tile t + PD is issued in the gaps of this tile's last MFMA phase (M2(B)), one piece per slot:
      // an LDS-DMA instruction stalls its wave ~90 cycles at issue (stamps: 462 cycles per tile for the five
      // pieces issued back to back after the barrier); behind an MFMA that stall runs under the matrix pipe
      const bool dma_next = t + C::PD < ntiles;
      const int DSLOT = (u + C::PD) % C::NBUF;  // a constant after unrolling
      KVP_SLOT();
      KVP_ST(2);
      const char* qs = smem + u * C::SLOT;
      const char* dos = qs + C::QIMG;
      const float* lsd = (const float*)(qs + 2 * C::QIMG);
      const bool diag = (CAUSAL && kw + 31 > q0cur) || kpad;        // half A has masked elements
      const bool diagB = (CAUSAL && kw + 31 > q0cur + 32) || kpad;  // half B has masked elements

      // The tile as 32 MFMA slots (one MFMA each, KVP_SLOT fences between them; every wait the compiler adds is a
      // counted lgkmcnt on reads issued two or more slots earlier):
      //   a1-a8 M1(A)  | Q / dO fragments of A and B, B's initial values
      //   b1-b8 M1(B)  | V(A) (one element pair per slot: 2 mul, 2 exp, 2 mul, 2 cvt_pk), A's transposed operands
      //   c1-c8 M2(A)  | V(A) tail, V(B), B's transposed operands
      //   d1-d8 M2(B)  | V(B) tail
      bf16x8 qa[KS], da[KS], qb[KS], db[KS];
      bf16x8 toA[2][DT], tqA[2][DT], toB[2][DT], tqB[2][DT];
      unsigned pwA[8], swA[8], pwB[8], swB[8];  // packed P / dS pairs: element pair e of a half -> word e
      auto vpair = [&](const f32x16& sv, const f32x16& dpv, int e, unsigned& pw, unsigned& sw)
          __attribute__((always_inline)) {
        typedef __attribute__((ext_vector_type(2))) float f32x2;
        typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
        const float p0 = fast_exp2(sv[2 * e] * c2), p1 = fast_exp2(sv[2 * e + 1] * c2);
        pw = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){p0, p1}, bf16x2));
        sw = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){p0 * dpv[2 * e], p1 * dpv[2 * e + 1]}, bf16x2));
      };
      auto pk4 = [&](const unsigned* w) __attribute__((always_inline)) {
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
        return __builtin_bit_cast(bf16x8, (u32x4){w[0], w[1], w[2], w[3]});
      };
      // A's operands and initial values (their latency is the one exposed read of the tile)
      qa[0] = lds_read_b128(qs, qo[0]);
      qa[1] = lds_read_b128(qs, qo[1]);
      f32x16 sA = init_rows(lsd, 0, 0);
      f32x16 dpA = init_rows(lsd, 0, 1);
      if (diag) mask_rows(sA, q0cur);
      f32x16 sB, dpB;
      KVP_SLOT();
      sA = mfma32(qa[0], kf[0], sA);  // a1
      qa[2] = lds_read_b128(qs, qo[2]);
      qa[3] = lds_read_b128(qs, qo[3]);
      KVP_SLOT();
      sA = mfma32(qa[1], kf[1], sA);  // a2
      da[0] = lds_read_b128(dos, qo[0]);
      da[1] = lds_read_b128(dos, qo[1]);
      KVP_SLOT();
      sA = mfma32(qa[2], kf[2], sA);  // a3
      da[2] = lds_read_b128(dos, qo[2]);
      da[3] = lds_read_b128(dos, qo[3]);
      KVP_SLOT();
      sA = mfma32(qa[3], kf[3], sA);  // a4
      sB = init_rows(lsd, 1, 0);
      KVP_SLOT();
      dpA = mfma32(da[0], vf[0], dpA);  // a5
      dpB = init_rows(lsd, 1, 1);
      KVP_SLOT();
      dpA = mfma32(da[1], vf[1], dpA);  // a6
      qb[0] = lds_read_b128(qs, qo[0] + 32 * RB);
      qb[1] = lds_read_b128(qs, qo[1] + 32 * RB);
      if (diagB) mask_rows(sB, q0cur + 32);
      KVP_SLOT();
      dpA = mfma32(da[2], vf[2], dpA);  // a7
      qb[2] = lds_read_b128(qs, qo[2] + 32 * RB);
      qb[3] = lds_read_b128(qs, qo[3] + 32 * RB);
      KVP_SLOT();
      dpA = mfma32(da[3], vf[3], dpA);  // a8
      db[0] = lds_read_b128(dos, qo[0] + 32 * RB);
      db[1] = lds_read_b128(dos, qo[1] + 32 * RB);
      KVP_SLOT();
      KVP_ST(3);
      sB = mfma32(qb[0], kf[0], sB);  // b1
      db[2] = lds_read_b128(dos, qo[2] + 32 * RB);
      db[3] = lds_read_b128(dos, qo[3] + 32 * RB);
      KVP_SLOT();
      sB = mfma32(qb[1], kf[1], sB);  // b2
      toA[0][0] = tr_pair(dos, tro[0][0], tro[0][1]);
      KVP_SLOT();
      sB = mfma32(qb[2], kf[2], sB);  // b3
      vpair(sA, dpA, 0, pwA[0], swA[0]);
      tqA[0][0] = tr_pair(qs, tro[0][0], tro[0][1]);
      KVP_SLOT();
      sB = mfma32(qb[3], kf[3], sB);  // b4
      vpair(sA, dpA, 1, pwA[1], swA[1]);
      toA[0][1] = tr_pair(dos, tro[1][0], tro[1][1]);
      KVP_SLOT();
      dpB = mfma32(db[0], vf[0], dpB);  // b5
      vpair(sA, dpA, 2, pwA[2], swA[2]);
      tqA[0][1] = tr_pair(qs, tro[1][0], tro[1][1]);
      KVP_SLOT();
      dpB = mfma32(db[1], vf[1], dpB);  // b6
      vpair(sA, dpA, 3, pwA[3], swA[3]);
      toA[1][0] = tr_pair(dos + 16 * RB, tro[0][0], tro[0][1]);
      KVP_SLOT();
      dpB = mfma32(db[2], vf[2], dpB);  // b7
      vpair(sA, dpA, 4, pwA[4], swA[4]);
      tqA[1][0] = tr_pair(qs + 16 * RB, tro[0][0], tro[0][1]);
      KVP_SLOT();
      dpB = mfma32(db[3], vf[3], dpB);  // b8
      vpair(sA, dpA, 5, pwA[5], swA[5]);
      toA[1][1] = tr_pair(dos + 16 * RB, tro[1][0], tro[1][1]);
      KVP_SLOT();
      KVP_ST(4);
      const bf16x8 pA0 = pk4(pwA), sA0 = pk4(swA);
      dv[0] = mfma32(toA[0][0], pA0, dv[0]);  // c1
      vpair(sA, dpA, 6, pwA[6], swA[6]);
      tqA[1][1] = tr_pair(qs + 16 * RB, tro[1][0], tro[1][1]);
      KVP_SLOT();
      dk[0] = mfma32(tqA[0][0], sA0, dk[0]);  // c2
      vpair(sA, dpA, 7, pwA[7], swA[7]);
      toB[0][0] = tr_pair(dos + 32 * RB, tro[0][0], tro[0][1]);
      KVP_SLOT();
      dv[1] = mfma32(toA[0][1], pA0, dv[1]);  // c3
      vpair(sB, dpB, 0, pwB[0], swB[0]);
      tqB[0][0] = tr_pair(qs + 32 * RB, tro[0][0], tro[0][1]);
      KVP_SLOT();
      dk[1] = mfma32(tqA[0][1], sA0, dk[1]);  // c4
      vpair(sB, dpB, 1, pwB[1], swB[1]);
      toB[0][1] = tr_pair(dos + 32 * RB, tro[1][0], tro[1][1]);
      KVP_SLOT();
      const bf16x8 pA1 = pk4(pwA + 4), sA1 = pk4(swA + 4);
      dv[0] = mfma32(toA[1][0], pA1, dv[0]);  // c5
      vpair(sB, dpB, 2, pwB[2], swB[2]);
      tqB[0][1] = tr_pair(qs + 32 * RB, tro[1][0], tro[1][1]);
      KVP_SLOT();
      dk[0] = mfma32(tqA[1][0], sA1, dk[0]);  // c6
      vpair(sB, dpB, 3, pwB[3], swB[3]);
      toB[1][0] = tr_pair(dos + 48 * RB, tro[0][0], tro[0][1]);
      KVP_SLOT();
      dv[1] = mfma32(toA[1][1], pA1, dv[1]);  // c7
      vpair(sB, dpB, 4, pwB[4], swB[4]);
      tqB[1][0] = tr_pair(qs + 48 * RB, tro[0][0], tro[0][1]);
      KVP_SLOT();
      dk[1] = mfma32(tqA[1][1], sA1, dk[1]);  // c8
      vpair(sB, dpB, 5, pwB[5], swB[5]);
      toB[1][1] = tr_pair(dos + 48 * RB, tro[1][0], tro[1][1]);
      KVP_SLOT();
      KVP_ST(5);
      const bf16x8 pB0 = pk4(pwB), sB0 = pk4(swB);
      dv[0] = mfma32(toB[0][0], pB0, dv[0]);  // d1
      vpair(sB, dpB, 6, pwB[6], swB[6]);
      tqB[1][1] = tr_pair(qs + 48 * RB, tro[1][0], tro[1][1]);
      KVP_SLOT();
      dk[0] = mfma32(tqB[0][0], sB0, dk[0]);  // d2
      vpair(sB, dpB, 7, pwB[7], swB[7]);
      KVP_SLOT();
      dv[1] = mfma32(toB[0][1], pB0, dv[1]);  // d3
      if (dma_next) issue_piece(DSLOT, nxt, 0);
      KVP_SLOT();
      dk[1] = mfma32(tqB[0][1], sB0, dk[1]);  // d4
      if (dma_next) issue_piece(DSLOT, nxt, 1);
      KVP_SLOT();
      const bf16x8 pB1 = pk4(pwB + 4), sB1 = pk4(swB + 4);
      dv[0] = mfma32(toB[1][0], pB1, dv[0]);  // d5
      if (dma_next) issue_piece(DSLOT, nxt, 2);
      KVP_SLOT();
      dk[0] = mfma32(tqB[1][0], sB1, dk[0]);  // d6
      if (PPW > 2 && dma_next) issue_piece(DSLOT, nxt, 3);
      KVP_SLOT();
      dv[1] = mfma32(toB[1][1], pB1, dv[1]);  // d7
      if (PPW > 2 && dma_next) issue_piece(DSLOT, nxt, 4);
      KVP_SLOT();
      dk[1] = mfma32(tqB[1][1], sB1, dk[1]);  // d8
      advance(nxt);
      KVP_SLOT();
      KVP_ST(6);
      q0cur = q0cur + QT2 >= qend ? qstart : q0cur + QT2;
    }
  }
#if PICO_KVP_STAMP
  tblk = __builtin_amdgcn_s_memtime();
#endif

  // ---- epilogue (as attn_bwd_kv_kernel): lane = key kw + r, register i of tile dt = d 32 dt + acc_row(i, h) ----
  if (hsplit == 1) {
    const int key = kw + r;
    const int kc = min(key, Sk - 1);
    if (a.flags & PICO_ATTN_ROPE_BWD) {
      const bf16_t* cp = (const bf16_t*)a.rope_cos + (int64_t)kc * a.rope_stride;
      const bf16_t* sp = (const bf16_t*)a.rope_sin + (int64_t)kc * a.rope_stride;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const u16x4 c4 = *reinterpret_cast<const u16x4*>(cp + 8 * g + 4 * h);
        const u16x4 s4 = *reinterpret_cast<const u16x4*>(sp + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float cf = bf2f(c4[j]), sn = bf2f(s4[j]);
          const float x1 = dk[0][4 * g + j], x2 = dk[1][4 * g + j];
          dk[0][4 * g + j] = x1 * cf + x2 * sn;
          dk[1][4 * g + j] = x2 * cf - x1 * sn;
        }
      }
    }
    bf16_t* dkp = (bf16_t*)a.dk + b * a.dk_strides[0] + hk * a.dk_strides[2] + (int64_t)kc * a.dk_strides[1];
    bf16_t* dvp = (bf16_t*)a.dv + b * a.dv_strides[0] + hk * a.dv_strides[2] + (int64_t)kc * a.dv_strides[1];
    store_row_bf16_x16<DT>(dkp, h, key < Sk, [&](int dt, int i) { return dk[dt][i] * scale; });
    store_row_bf16_x16<DT>(dvp, h, key < Sk, [&](int dt, int i) { return dv[dt][i]; });
  } else {  // fp32 partials [hs][dK | dV][b][key][hk][D]
    const int64_t part = a.batch * a.seqlen_k * a.heads_kv * 64;
    float* pk = dkv_part + (int64_t)(2 * hs) * part + ((int64_t)b * Sk * a.heads_kv + hk) * 64;
    float* pv = pk + part;
    const int key = kw + r;
    if (key < Sk) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 wk, wv;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            wk[j] = dk[dt][4 * g + j] * scale;
            wv[j] = dv[dt][4 * g + j];
          }
          const int64_t o = (int64_t)key * a.heads_kv * 64 + 32 * dt + 8 * g + 4 * h;
          *reinterpret_cast<f32x4*>(pk + o) = wk;
          *reinterpret_cast<f32x4*>(pv + o) = wv;
        }
    }
  }
#if PICO_KVP_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ph[9] += __builtin_amdgcn_s_memtime() - tblk;  // epilogue of this block (stores drained)
#endif
  }  // key blocks of the group
#if PICO_KVP_STAMP
  ph[11] = __builtin_amdgcn_s_memrealtime();
  ph[13] = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0 && (int64_t)blockIdx.x * NW + wave < STAMP_BYTES / 128) {
#pragma unroll
    for (int i = 0; i < 16; ++i) stamp_out[((int64_t)blockIdx.x * NW + wave) * 16 + i] = ph[i];
  }
#endif
}
#undef KVP_ST
#undef KVP_SLOT

// attn_bwd_kvp_kernel (64-row tiles) for D = 64 up to 1536 causal / 4096 non-causal keys, the 32-row kernel beyond.
// Same box, 3 interleaved rounds each (profiles/r05_ab_kvp_default.jsonl, r05_ab_kvp_long.jsonl,
// r05_ab_kvp_waves.jsonl): dK/dV C2 55.2 -> 53.5 us, GQA-4 57.4 -> 53.2, C2 non-causal 76.7 -> 72.7, S 4096
// non-causal (config 5's off-diagonal ring blocks) 266.7 -> 255.5; at S 2048 causal the two kernels measured equal
// on one box (81.3 vs 81.0) and 91.0 vs 95.7 on another, at S 4096 causal 138.5 vs 144.7 and 143.7 vs 150.6.
// pico_select(PICO_SEL_ATTN_KVP, 0 / 1) forces either (A/B switch).
bool kvp_enabled(const pico_attn_args* a) {
  if (a->head_dim != 64) return false;
  const int e = pico_sel(PICO_SEL_ATTN_KVP);
  if (e != PICO_SEL_AUTO) return e != 0;
  return a->seqlen_k <= (a->causal ? 1536 : 4096);
}

// waves (x 32 keys) per attn_bwd_kvp_kernel workgroup: 4 (two 128-key workgroups per CU), or 8 (one 256-key
// workgroup per CU: each Q / dO tile loaded and each barrier taken once for twice the keys) for non-causal blocks of
// 2048 keys and more: S 4096 non-causal 259.8 -> 256.8 us; at C2 shapes 8 waves lose (C2 52.9 -> 57.9, GQA-4
// 53.1 -> 65.5: a 256-workgroup grid is too coarse there). pico_select(PICO_SEL_KVP_WAVES, 4 / 8) forces either.
int kvp_waves(const pico_attn_args* a) {
  const int e = pico_sel(PICO_SEL_KVP_WAVES);
  if (e == 4 || e == 8) return e;
  return !a->causal && a->seqlen_k >= 2048 ? 8 : 4;
}

#endif  // !PICO_SPLIT_D128_TU

#ifdef PICO_SPLIT_D128_TU
// ------------------------------------------------------------------------------------------------
// dK / dV kernel, D = 128, 64-row query tiles in a slot-ordered stream (round 6)
// ------------------------------------------------------------------------------------------------
// attn_bwd_kvp_kernel's form carried to head_dim 128: a workgroup = 4 waves x 32 keys (dK / dV of the wave's keys
// in 128 accumulator registers, K / V fragments resident), each ring tile 64 query rows as halves A / B whose
// phases interleave inside the wave:
//     M1(A) | A's then B's Q / dO operands,  M1(B) | V(A) + A's transposed reads,  M2(A) | V(B) + B's reads,
//     M2(B) | the DMA of tile t + 2
// 16 MFMAs per phase (64 per tile: at D = 128 the tile is MFMA-bound, ~130 VALU against 2,048 matrix cycles), one
// wave per SIMD (the whole register file: dK / dV and K / V in AGPRs, the S / dP pipeline in VGPRs; one 99-KiB
// workgroup per CU). The 32-row kernel it replaces runs each
// 32-row tile as one dependency chain (S / dP -> softmax -> dV / dK) at one wave per SIMD: 0.22 MFMA busy at C4.
// Operands are read two slots ahead of their MFMA; the schedule is fenced per slot (sched_barrier).
constexpr int QT2 = 64;  // query rows per ring tile (the D = 64 TU defines it with attn_bwd_kvp_kernel)
struct KV2Cfg {
  static constexpr int D = 128, KS = 8, DT = 4;
  static constexpr int QIMG = QT2 * 256;         // one Q (or dO) 64-row image (kv2_off), 16 KiB
  static constexpr int LSD = 1024;               // -LSE/scale [64] | -delta [64] (+ 512 B the DMA piece repeats)
  static constexpr int SLOT = 2 * QIMG + LSD;    // 33 KiB
  // 99 KiB per workgroup, prefetch distance 2 (a 4-deep ring measured 1-5 % slower)
  static constexpr int NBUF = 3, PD = NBUF - 1;
  static constexpr int NQP = QIMG / 1024;        // 16 pieces per image
  static constexpr int PPW = 2 * NQP / 4;        // 8 image pieces per wave per tile (+ wave 0's LSE / delta piece)
};

#define KV2_SLOT() __builtin_amdgcn_sched_barrier(0)

// byte offset of 16-byte chunk ch (0..15) of row `row` in a [64][128 x bf16] image of 8-row x 32-column subtiles of
// 512 B (cdna_hip_programming.md T11 image (a)): the row reads of a k-step parity and the transposed reads of a row
// parity share one base register each (every other offset an immediate), both conflict-free
PICO_DEV int kv2_off(int row, int ch) {
  return 2048 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

template <bool CAUSAL>
__global__ __launch_bounds__(256, 1) void attn_bwd_kvp128_kernel(const pico_attn_args a, float scale, float c2,
                                                                 const float* __restrict__ sinit_g,
                                                                 const float* __restrict__ delta_g, int sq_pad,
                                                                 int hsplit, float* __restrict__ dkv_part,
                                                                 const BlkGroups grp,
                                                                 unsigned long long* __restrict__ stamp_out) {
  using C = KV2Cfg;
#if PICO_KVP_STAMP  // the stamp words of attn_bwd_kvp_kernel (scripts/kvp_stamps.py): 0 wait, 1 barrier, 3-6 phases
  unsigned long long ph[16] = {0}, tlast = 0, tblk = 0;
  ph[10] = __builtin_amdgcn_s_memrealtime();
  ph[12] = __builtin_amdgcn_s_memtime();
#define KV2_ST(i)                                               \
  {                                                             \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    ph[i] += t_ - tlast;                                        \
    tlast = t_;                                                 \
  }
#else
#define KV2_ST(i)
#endif
  constexpr int KS = C::KS, DT = C::DT, PPW = C::PPW, NW = 4, KB = 32 * NW;
  // M1 operands are read RD slots ahead of their MFMA (3 vs 2: 0.7-1.4 % less time at C4 / non-causal / GQA-4 over
  // 2 x 2 rounds, profiles/r06_kvp128_rd/; 4 no better)
  constexpr int RD = 3;
  static_assert(PPW == 8 && 2 * C::NQP == PPW * NW, "8 image pieces per wave: the odd slots of M2(B)");
  __shared__ __attribute__((aligned(16))) char smem[C::NBUF * C::SLOT];

  const int lane0 = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int Sq = (int)a.seqlen_q, Sk = (int)a.seqlen_k;
  const int Hq = (int)a.heads_q;
  const int G = (int)(a.heads_q / a.heads_kv);
  const int nbh = (int)(a.batch * a.heads_kv) * hsplit;
  const int gi = blockIdx.x / nbh;
  const int bhs = blockIdx.x % nbh;
  const int hs = bhs % hsplit;
  const int bh = bhs / hsplit;
  const int b = bh / (int)a.heads_kv, hk = bh % (int)a.heads_kv;
  const unsigned gw = grp.n ? grp_sel(grp, gi) : 0u;
  const int nblk_wg = grp.n ? (int)((grp.cnt >> (4 * gi)) & 15ull) : 1;
  const unsigned delta_off = (unsigned)((const char*)delta_g - (const char*)sinit_g);  // same workspace
  const unsigned ring_lds = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr(smem));
#pragma clang loop unroll(disable)
  for (int jb = 0; jb < nblk_wg; ++jb) {
#if PICO_KVP_STAMP
    tblk = __builtin_amdgcn_s_memtime();
#endif
    const int kb = grp.n ? (int)((gw >> (8 * jb)) & 255u) : gi;
    if (jb > 0) lds_barrier();
    int lane_l = lane0;
    asm volatile("" : "+v"(lane_l));
    const int lane = lane_l, r = lane & 31, h = lane >> 5;
    const int k0 = kb * KB;
    const int kw = k0 + 32 * wave;
    const int qstart = CAUSAL ? k0 : 0;  // k0 is a multiple of QT2
    const int nqt = Sq > qstart ? (Sq - qstart + QT2 - 1) / QT2 : 0;
    const int ntot = G * nqt;
    const int tb = (int)((int64_t)ntot * hs / hsplit);
    const int ntiles = (int)((int64_t)ntot * (hs + 1) / hsplit) - tb;
    const int hq0 = hk * G + (nqt ? tb / nqt : 0), q00 = qstart + (nqt ? tb % nqt : 0) * QT2;

    // ---- tile DMA: this wave's image pieces i = 0..PPW-1 (Q: i < PPW/2, dO after) are image pieces
    // (wave + 4 i) % NQP; wave 0 also issues the LSE / delta piece ----
    const int64_t qs1 = a.q_strides[1] * 2, ds1 = a.do_strides[1] * 2;  // bytes per query row
    const char* const qbase = (const char*)((const bf16_t*)a.q + b * a.q_strides[0]);
    const char* const dobase = (const char*)((const bf16_t*)a.dout + b * a.do_strides[0]);
    // piece jj of an image = LDS bytes [1024 jj, 1024 jj + 1024): lane l lands 16 bytes at 1024 jj + 16 l, i.e. row
    // 8 (jj >> 1) + ((l & 31) >> 2), chunk 4 (2 (jj & 1) + (l >> 5)) + ((l & 3) ^ ((row >> 2) & 3)) of kv2_off
    auto piece_row = [&](int jj, int l) __attribute__((always_inline)) { return 8 * (jj >> 1) + ((l & 31) >> 2); };
    auto piece_ch = [&](int jj, int l, int row) __attribute__((always_inline)) {
      return 4 * (2 * (jj & 1) + (l >> 5)) + ((l & 3) ^ ((row >> 2) & 3));
    };
    unsigned pc_off[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int jj = (wave + 4 * i) % C::NQP;
      const int row = piece_row(jj, lane);
      pc_off[i] = (unsigned)(row * (i < PPW / 2 ? qs1 : ds1) + 16 * piece_ch(jj, lane, row));
    }
    struct Tc {
      int hq, q0;
      const char* qp;
      const char* dp;
      const char* lp;
    };
    auto make_tc = [&](int hq, int q0) __attribute__((always_inline)) {
      Tc c;
      c.hq = hq;
      c.q0 = q0;
      c.qp = qbase + hq * a.q_strides[2] * 2 + q0 * qs1;
      c.dp = dobase + hq * a.do_strides[2] * 2 + q0 * ds1;
      c.lp = (const char*)(sinit_g + ((int64_t)b * Hq + hq) * sq_pad + q0);
      return c;
    };
    const int qend = qstart + nqt * QT2;
    auto advance = [&](Tc& c) __attribute__((always_inline)) {
      if (c.q0 + QT2 >= qend) {
        c = make_tc(c.hq + 1, qstart);
      } else {
        c.q0 += QT2;
        c.qp += QT2 * qs1;
        c.dp += QT2 * ds1;
        c.lp += QT2 * 4;
      }
    };
    const bool ragged = Sq % QT2 != 0;
    auto issue_piece = [&](int si, const Tc& c, int i) __attribute__((always_inline)) {
      const unsigned dst = ring_lds + (unsigned)si * (unsigned)C::SLOT;
      if (i < PPW) {
        const int jj = (wave + 4 * i) % C::NQP;
        unsigned off = pc_off[i];
        if (ragged && c.q0 + QT2 > Sq) {  // partial tile: rows past Sq - 1 clamped (finite; their LSE is +inf)
          int l2 = lane0;
          asm volatile("" : "+v"(l2));
          const int row = piece_row(jj, l2 & 63);
          off = (unsigned)((min(c.q0 + row, Sq - 1) - c.q0) * (i < PPW / 2 ? qs1 : ds1) +
                           16 * piece_ch(jj, l2 & 63, row));
        }
        dma_piece(i < PPW / 2 ? c.qp : c.dp, off, dst + (i < PPW / 2 ? 0u : (unsigned)C::QIMG) + (unsigned)jj * 1024u);
      } else if (wave == 0) {
        int l = lane0;
        asm volatile("" : "+v"(l));
        l &= 31;
        dma_piece(c.lp, (unsigned)(16 * (l & 15)) + ((l >> 4) ? delta_off : 0u), dst + 2u * C::QIMG);
      }
    };
    Tc nxt = make_tc(hq0, q00);
#pragma unroll
    for (int j = 0; j < C::PD; ++j) {
      if (j < ntiles) {
#pragma unroll
        for (int i = 0; i <= PPW; ++i) issue_piece(j, nxt, i);
      }
      advance(nxt);
    }

    // ---- K, V fragments of this wave's 32 keys (B operands of S and dP) ----
    const bf16_t* kg = (const bf16_t*)a.k + b * a.k_strides[0] + hk * a.k_strides[2];
    const bf16_t* vg = (const bf16_t*)a.v + b * a.v_strides[0] + hk * a.v_strides[2];
    bf16x8 kf[KS], vf[KS];
    {
      const int key = kw + r;
      const bool ok = key < Sk;
      const bf16_t* kp = kg + (int64_t)min(key, Sk - 1) * a.k_strides[1] + 8 * h;
      const bf16_t* vp = vg + (int64_t)min(key, Sk - 1) * a.v_strides[1] + 8 * h;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const u16x8 kv = *reinterpret_cast<const u16x8*>(kp + 16 * ks);
        const u16x8 vv = *reinterpret_cast<const u16x8*>(vp + 16 * ks);
        kf[ks] = __builtin_bit_cast(bf16x8, ok ? kv : (u16x8)0);
        vf[ks] = __builtin_bit_cast(bf16x8, ok ? vv : (u16x8)0);
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      asm volatile("" : "+a"(kf[ks]), "+a"(vf[ks]));  // resident in AGPRs: the MFMAs take their B operand there
    }
    f32x16 dk[DT], dv[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      dk[dt] = (f32x16)0.f;
      dv[dt] = (f32x16)0.f;
      asm volatile("" : "+a"(dk[dt]), "+a"(dv[dt]));
    }
    // row-read bases by k-step parity (k-step ks adds 512 (ks >> 1), half X 8192), transposed-read bases of rows
    // 4 hh + q and + 8 (tile dt adds 512 dt, 16-row step st 4096 st, half X 8192)
    unsigned qo[2], tro[2];
    {
      const int g = lane >> 4, i = lane & 15, hh = g >> 1, q = i >> 2, p = i & 3;
      qo[0] = kv2_off(r, h);
      qo[1] = kv2_off(r, 2 + h);
      tro[0] = kv2_off(4 * hh + q, 2 * (g & 1) + (p >> 1)) + 8 * (p & 1);
      tro[1] = kv2_off(4 * hh + q + 8, 2 * (g & 1) + (p >> 1)) + 8 * (p & 1);
    }
    const bool kpad = kw + 31 >= Sk;  // wave-uniform: some of the wave's keys are padding
    const int mykey = kw + r;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#if PICO_KVP_STAMP
    ph[8] += __builtin_amdgcn_s_memtime() - tblk;
#endif

    auto init_rows = [&](const float* lsd, int X, int which) __attribute__((always_inline)) {
      f32x16 v;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 t4 = *reinterpret_cast<const f32x4*>(lsd + 64 * which + 32 * X + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[4 * g + j] = t4[j];
      }
      return v;
    };
    auto mask_rows = [&](f32x16& sv, int qrow0) __attribute__((always_inline)) {
      const int rel = mykey >= Sk ? 1 << 30 : (CAUSAL ? mykey - qrow0 - 4 * h : -1);
#pragma unroll
      for (int i = 0; i < 16; ++i) sv[i] = ((i & 3) + 8 * (i >> 2) < rel) ? -INFINITY : sv[i];
    };
    auto vpair = [&](const f32x16& sv, const f32x16& dpv, int e, unsigned& pw, unsigned& sw) __attribute__((always_inline)) {
      typedef __attribute__((ext_vector_type(2))) float f32x2;
      typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
      const float p0 = fast_exp2(sv[2 * e] * c2), p1 = fast_exp2(sv[2 * e + 1] * c2);
      pw = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){p0, p1}, bf16x2));
      sw = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){p0 * dpv[2 * e], p1 * dpv[2 * e + 1]}, bf16x2));
    };
    auto pk4 = [&](const unsigned* w) __attribute__((always_inline)) {
      typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
      return __builtin_bit_cast(bf16x8, (u32x4){w[0], w[1], w[2], w[3]});
    };

    int q0cur = q00;
    for (int t0 = 0; t0 < ntiles; t0 += C::NBUF) {  // unrolled by the ring depth: slot offsets are immediates
#pragma unroll
    for (int u = 0; u < C::NBUF; ++u) {
      const int t = t0 + u;
      if (t >= ntiles) break;
#if PICO_KVP_STAMP
      tlast = __builtin_amdgcn_s_memtime();
      ph[7] += 1;
#endif
      if (t > 0) {
        // this wave's pieces of tile t landed; those of the younger tiles already issued stay in flight
        const int younger = min(C::PD - 1, ntiles - 1 - t);
        if (younger >= 2 && C::PD >= 3) {
          if (wave == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (PPW + 1)) : "memory");
          else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PPW) : "memory");
        } else if (younger >= 1) {
          if (wave == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW + 1) : "memory");
          else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPW) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        KV2_ST(0);
        lds_barrier();  // every wave's pieces of tile t visible; the slot of tile t - 1 is no longer read
        KV2_ST(1);
      }
      const bool dma_next = t + C::PD < ntiles;
      const int dslot = (u + C::PD) % C::NBUF;  // a constant after unrolling
      const char* qs = smem + u * C::SLOT;
      const char* dos = qs + C::QIMG;
      const float* lsd = (const float*)(qs + 2 * C::QIMG);
      const bool diag = (CAUSAL && kw + 31 > q0cur) || kpad;        // half A has masked elements
      const bool diagB = (CAUSAL && kw + 31 > q0cur + 32) || kpad;  // half B has masked elements
      KV2_SLOT();

      // M1 operands of half X, read in slot order: [Q k-steps 0..KS-1, dO k-steps 0..KS-1]
      bf16x8 opA[2 * KS], opB[2 * KS];
      auto rd_op = [&](bf16x8 (&op)[2 * KS], int X, int k) __attribute__((always_inline)) {
        op[k] = lds_read_b128((k < KS ? qs : dos) + 512 * ((k % KS) >> 1) + 8192 * X, qo[k & 1]);
      };
      // M2 operands of half X: [st][dt] -> (dO^T, Q^T) pairs, read in slot order k = 2 (DT st + dt) + {0: dO^T, 1: Q^T}
      bf16x8 toA[2][DT], tqA[2][DT], toB[2][DT], tqB[2][DT];
      auto rd_tr = [&](bf16x8 (&to)[2][DT], bf16x8 (&tq)[2][DT], int X, int k) __attribute__((always_inline)) {
        const int st = k / (2 * DT), dt = (k / 2) % DT;
        const char* base = ((k & 1) ? qs : dos) + 8192 * X + 4096 * st + 512 * dt;
        if (k & 1) tq[st][dt] = tr_pair(base, tro[0], tro[1]);
        else to[st][dt] = tr_pair(base, tro[0], tro[1]);
      };
      unsigned pwA[8], swA[8], pwB[8], swB[8];

      // ---- M1(A): S_A (k < KS), dP_A (k >= KS); operands two slots ahead; B's first operands + initial values ----
      f32x16 sA = init_rows(lsd, 0, 0), dpA = init_rows(lsd, 0, 1);
      if (diag) mask_rows(sA, q0cur);
      static_for<RD>([&](auto k_) { rd_op(opA, 0, decltype(k_)::value); });
      f32x16 sB, dpB;
      KV2_SLOT();
      static_for<2 * KS>([&](auto k_) {
        constexpr int k = decltype(k_)::value;
        if constexpr (k < KS) sA = mfma32(opA[k], kf[k], sA);
        else dpA = mfma32(opA[k], vf[k - KS], dpA);
        if constexpr (k + RD < 2 * KS) rd_op(opA, 0, k + RD);
        else rd_op(opB, 1, k + RD - 2 * KS);
        if constexpr (k == 4) sB = init_rows(lsd, 1, 0);
        if constexpr (k == 6) dpB = init_rows(lsd, 1, 1);
        if constexpr (k == 8) {
          if (diagB) mask_rows(sB, q0cur + 32);
        }
        KV2_SLOT();
      });
      KV2_ST(3);
      // ---- M1(B): S_B, dP_B | V(A) (one element pair per two slots) + A's transposed operands (one per slot) ----
      static_for<2 * KS>([&](auto k_) {
        constexpr int k = decltype(k_)::value;
        if constexpr (k < KS) sB = mfma32(opB[k], kf[k], sB);
        else dpB = mfma32(opB[k], vf[k - KS], dpB);
        if constexpr (k + RD < 2 * KS) rd_op(opB, 1, k + RD);
        if constexpr ((k & 1) == 0) vpair(sA, dpA, k / 2, pwA[k / 2], swA[k / 2]);
        rd_tr(toA, tqA, 0, k);
        KV2_SLOT();
      });
      KV2_ST(4);
      // ---- M2(A): dV^T += dO^T P, dK^T += Q^T dS over A's rows | V(B) + B's transposed operands ----
      {
        const bf16x8 pA[2] = {pk4(pwA), pk4(pwA + 4)}, sAp[2] = {pk4(swA), pk4(swA + 4)};
        static_for<2 * KS>([&](auto k_) {
          constexpr int k = decltype(k_)::value;
          constexpr int st = k / (2 * DT), dt = (k / 2) % DT;
          if constexpr ((k & 1) == 0) mfma32_acc(dv[dt], toA[st][dt], pA[st]);
          else mfma32_acc(dk[dt], tqA[st][dt], sAp[st]);
          if constexpr ((k & 1) == 0) vpair(sB, dpB, k / 2, pwB[k / 2], swB[k / 2]);
          rd_tr(toB, tqB, 1, k);
          KV2_SLOT();
        });
      }
      KV2_ST(5);
      // ---- M2(B) | the DMA of tile t + 2 ----
      {
        const bf16x8 pB[2] = {pk4(pwB), pk4(pwB + 4)}, sBp[2] = {pk4(swB), pk4(swB + 4)};
        static_for<2 * KS>([&](auto k_) {
          constexpr int k = decltype(k_)::value;
          constexpr int st = k / (2 * DT), dt = (k / 2) % DT;
          if constexpr ((k & 1) == 0) mfma32_acc(dv[dt], toB[st][dt], pB[st]);
          else mfma32_acc(dk[dt], tqB[st][dt], sBp[st]);
          if constexpr ((k & 1) == 1) {  // image pieces 0..7 in the odd slots (measured: 2, 4 or all 8 of them
            if (dma_next) issue_piece(dslot, nxt, k / 2);  // in M2(A)'s slots instead is 0-3 % slower)
          } else if constexpr (k == 0) {  // the LSE / delta piece
            if (dma_next) issue_piece(dslot, nxt, PPW);
          }
          KV2_SLOT();
        });
      }
      KV2_ST(6);
      advance(nxt);
      q0cur = q0cur + QT2 >= qend ? qstart : q0cur + QT2;
    }
    }
    // the last accumulations complete (32x32 MFMA write -> read: up to 18 wait states) before the epilogue reads them
    acc_drain4(dk);
    acc_drain4(dv);
#if PICO_KVP_STAMP
    const unsigned long long tep = __builtin_amdgcn_s_memtime();
#endif

    // ---- epilogue: lane = key kw + r, register i of tile dt = d 32 dt + acc_row(i, h) ----
    if (hsplit == 1) {
      const int key = kw + r;
      const int kc = min(key, Sk - 1);
      if (a.flags & PICO_ATTN_ROPE_BWD) {  // rotate back by -theta: pairs (d, d + D/2) = tiles (dt, dt + DT/2)
        const bf16_t* cp = (const bf16_t*)a.rope_cos + (int64_t)kc * a.rope_stride;
        const bf16_t* sp = (const bf16_t*)a.rope_sin + (int64_t)kc * a.rope_stride;
#pragma unroll
        for (int dt = 0; dt < DT / 2; ++dt)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const u16x4 c4 = *reinterpret_cast<const u16x4*>(cp + 32 * dt + 8 * g + 4 * h);
            const u16x4 s4 = *reinterpret_cast<const u16x4*>(sp + 32 * dt + 8 * g + 4 * h);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float cf = bf2f(c4[j]), sn = bf2f(s4[j]);
              const float x1 = dk[dt][4 * g + j], x2 = dk[dt + DT / 2][4 * g + j];
              dk[dt][4 * g + j] = x1 * cf + x2 * sn;
              dk[dt + DT / 2][4 * g + j] = x2 * cf - x1 * sn;
            }
          }
      }
      bf16_t* dkp = (bf16_t*)a.dk + b * a.dk_strides[0] + hk * a.dk_strides[2] + (int64_t)kc * a.dk_strides[1];
      bf16_t* dvp = (bf16_t*)a.dv + b * a.dv_strides[0] + hk * a.dv_strides[2] + (int64_t)kc * a.dv_strides[1];
      store_row_bf16_x16<DT>(dkp, h, key < Sk, [&](int dt, int i) { return dk[dt][i] * scale; });
      store_row_bf16_x16<DT>(dvp, h, key < Sk, [&](int dt, int i) { return dv[dt][i]; });
    } else {  // fp32 partials [hs][dK | dV][b][key][hk][D]
      const int64_t part = a.batch * a.seqlen_k * a.heads_kv * 128;
      float* pk = dkv_part + (int64_t)(2 * hs) * part + ((int64_t)b * Sk * a.heads_kv + hk) * 128;
      float* pv = pk + part;
      const int key = kw + r;
      if (key < Sk) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            f32x4 wk, wv;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              wk[j] = dk[dt][4 * g + j] * scale;
              wv[j] = dv[dt][4 * g + j];
            }
            const int64_t o = (int64_t)key * a.heads_kv * 128 + 32 * dt + 8 * g + 4 * h;
            *reinterpret_cast<f32x4*>(pk + o) = wk;
            *reinterpret_cast<f32x4*>(pv + o) = wv;
          }
      }
    }
#if PICO_KVP_STAMP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ph[9] += __builtin_amdgcn_s_memtime() - tep;
#endif
  }  // key blocks of the group
#if PICO_KVP_STAMP
  ph[11] = __builtin_amdgcn_s_memrealtime();
  ph[13] = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0 && (int64_t)blockIdx.x * 4 + wave < STAMP_BYTES / 128) {
#pragma unroll
    for (int i = 0; i < 16; ++i) stamp_out[((int64_t)blockIdx.x * 4 + wave) * 16 + i] = ph[i];
  }
#else
  (void)stamp_out;
#endif
}
#undef KV2_SLOT
#undef KV2_ST

// attn_bwd_kvp128_kernel for head_dim 128 (pico_select(PICO_SEL_ATTN_KVP, 0 / 1) forces the 32-row kernel or it)
bool kvp128_enabled(const pico_attn_args* a) {
  if (a->head_dim != 128) return false;
  const int e = pico_sel(PICO_SEL_ATTN_KVP);
  if (e != PICO_SEL_AUTO) return e != 0;
  return true;
}
#endif  // PICO_SPLIT_D128_TU

// keys per dK/dV workgroup block
int kv_block(const pico_attn_args* a) {
#ifndef PICO_SPLIT_D128_TU
  if (kvp_enabled(a)) return 32 * kvp_waves(a);
#endif
  (void)a;
  return KVB;
}

// rows of the LSE / delta workspace per (batch, head): padded to the 64-row tiles of attn_bwd_kvp_kernel
int split_sq_pad(const pico_attn_args* a) { return (int)((a->seqlen_q + 63) / 64) * 64; }

int64_t split_lsd_floats(const pico_attn_args* a) {
  const int64_t n = a->batch * a->heads_q * (int64_t)split_sq_pad(a);
  return ((n + 63) / 64) * 64;
}

// dK/dV workgroups per CU the register budget is sized for: 3 (168 VGPRs) for causal grids, whose LPT-ordered
// uneven blocks fill any number of slots (C2 58.5 -> 52.6 us, S 4096 153 -> 143); 2 (256 VGPRs) for non-causal
// grids, whose equal blocks would leave a third round partly empty (C2 full: 1024 blocks = 2 rounds of 512 slots
// vs 1.33 rounds of 768) and whose mask-free body spills at 168 VGPRs (83 vs 123 us); 1 at D = 128 (≈ 340
// registers: its own translation unit, AGPRs allowed).
int kv_minb(const pico_attn_args* a) {
  if (a->head_dim == 128) return 1;
#ifndef PICO_SPLIT_D128_TU
  if (kvp_enabled(a)) return kvp_waves(a) == 8 ? 1 : 2;  // attn_bwd_kvp_kernel: two waves per SIMD, <= 256 VGPRs
#endif
  return a->causal ? 3 : 2;
}

// split of a key block's tile list so that the dK/dV grid fills the 256 CUs (kv_minb workgroups each; GQA-4
// C2 at MINB 3: kv + dkv 55.5 + 13.8 us with 4 parts, 67.2 + 9.6 with 2, 62.1 + 9.7 at MINB 2)
int kv_hsplit(const pico_attn_args* a) {
  if (a->heads_kv <= 0 || a->heads_q % a->heads_kv != 0) return 1;
  const int kvb = kv_block(a);
  const int64_t nblk = ((a->seqlen_k + kvb - 1) / kvb) * a->batch * a->heads_kv;
  const int64_t tiles = (a->heads_q / a->heads_kv) * ((a->seqlen_q + QT - 1) / QT);
  if (nblk <= 0) return 1;
  int d = 1;
  while (d < 8 && nblk * d < 256 * kv_minb(a) && 2 * d <= tiles) d *= 2;
  return d;
}

}  // namespace
int64_t pico_attn_bwd_split_workspace(const pico_attn_args* a);
namespace {

// dQ kernel: query blocks dispatched lightest-first (see attn_bwd_q_kernel)
int q_front(const pico_attn_args* a) {
  if (!a->causal) return 0;
  const int nmb = (int)((a->seqlen_q + QB - 1) / QB);
  const int64_t nbh = a->batch * a->heads_q;
  const int minb = a->head_dim == 64 ? QCfg<64>::MINB : QCfg<128>::MINB;
  const int64_t first = (int64_t)pico_num_cus() * minb / (nbh > 0 ? nbh : 1);  // groups resident at once
  return first < nmb ? (int)(nmb - first) : 0;
}

// pico_select(PICO_SEL_ATTN_GROUPS, 0) restores the plain causal grids (one block per workgroup; A/B switch)
bool groups_enabled() { return pico_sel(PICO_SEL_ATTN_GROUPS) != 0; }

// The one-round schedule of BlkGroups: the nblk blocks of each (batch, head) (work wt[i] in tiles) cut into
// G = minb * CUs / nbh groups, so that the grid is exactly one round of minb workgroups per CU. Groups are
// dispatched g-major, so a group's place among a CU's resident workgroups (oldest first) is g * nbh / CUs; its
// target work is proportional to the tile rate of that place (measured at three per CU, C2 dK/dV: 1.15 / 1.53 /
// 2.2 us per tile -> 1 / 0.75 / 0.53). Blocks go heaviest first to the group with the most target left (at most
// 4 per group). n = 0 (the plain grid) when that grid is one round already or the cut does not fit the table.
BlkGroups block_groups(const int* wt, int nblk, int64_t nbh, int minb) {
  BlkGroups t{};
  const int cus = pico_num_cus();
  const int64_t slots = (int64_t)minb * cus;
  if (!groups_enabled() || nbh <= 0 || nblk > 32 || (int64_t)nblk * nbh <= slots) return t;
  const int G = (int)(slots / nbh);
  if (G < 2 || G > GRP_MAX || nblk > 4 * G) return t;
  static const double spd[3] = {1.0, 0.75, 0.53};
  double tgt[GRP_MAX], load[GRP_MAX] = {0.0}, tot = 0.0, ssum = 0.0;
  int cnt[GRP_MAX] = {0};
  for (int i = 0; i < nblk; ++i) tot += wt[i];
  for (int g = 0; g < G; ++g) {
    const int cls = (int)std::min<int64_t>(minb - 1, (int64_t)g * nbh / cus);
    tgt[g] = minb == 1 ? 1.0 : spd[std::min(cls, 2)];
    ssum += tgt[g];
  }
  for (int g = 0; g < G; ++g) tgt[g] *= tot / ssum;
  int order[32];
  for (int i = 0; i < nblk; ++i) order[i] = i;
  std::stable_sort(order, order + nblk, [&](int x, int y) { return wt[x] > wt[y]; });
  for (int k = 0; k < nblk; ++k) {
    const int i = order[k];
    int best = -1;
    for (int g = 0; g < G; ++g)
      if (cnt[g] < 4 && (best < 0 || tgt[g] - load[g] > tgt[best] - load[best])) best = g;
    if (best < 0) return BlkGroups{};
    t.w[best] |= (unsigned)i << (8 * cnt[best]);
    ++cnt[best];
    load[best] += wt[i];
  }
  for (int g = 0; g < G; ++g) {
    if (cnt[g] == 0) return BlkGroups{};
    t.cnt |= (unsigned long long)cnt[g] << (4 * g);
  }
  t.n = G;
  return t;
}

// dK/dV kernel groups: key block kb sees (Hq / Hkv) * ceil((Sq - 128 kb) / 32) query tiles (causal, no hsplit)
BlkGroups kv_groups(const pico_attn_args* a, int hsplit, int minb) {
  if (!a->causal || hsplit != 1 || a->heads_kv <= 0) return BlkGroups{};
  const int kvb = kv_block(a);
  const int nkb = (int)((a->seqlen_k + kvb - 1) / kvb);
  if (nkb > 32) return BlkGroups{};
  int wt[32];
  for (int kb = 0; kb < nkb; ++kb) {
    const int64_t q0 = (int64_t)kb * kvb;
    wt[kb] = (int)((a->heads_q / a->heads_kv) * (a->seqlen_q > q0 ? (a->seqlen_q - q0 + QT - 1) / QT : 0));
  }
  return block_groups(wt, nkb, a->batch * a->heads_kv, minb);
}

template <int D, bool CAUSAL>
int launch_split(const pico_attn_args* a, hipStream_t s) {
  const int sq_pad = split_sq_pad(a);
  float* lse2 = (float*)a->workspace;
  float* delta = lse2 + split_lsd_floats(a);
  float* dkv_part = delta + split_lsd_floats(a);
  const float sl2 = a->softmax_scale * LOG2E;
#ifndef PICO_SPLIT_D128_TU
  const bool use_kvp = D == 64 && kvp_enabled(a);
#else
  const bool use_kvp = D == 128 && kvp128_enabled(a);  // attn_bwd_kvp128_kernel: the -LSE/scale workspace form
#endif
  const int nmb = (int)((a->seqlen_q + QB - 1) / QB);
  const int64_t gq = (int64_t)nmb * a->batch * a->heads_q;
  PICO_REQUIRE(gq < (1ll << 31), "pico_attn_bwd: grid too large");
  PICO_TRY(pico_launch(PICO_K_ATTN_BWD_Q, "attn_bwd_q", attn_bwd_q_kernel<D, CAUSAL>, dim3((int)gq), dim3(256), 0, s,
                       *a, a->softmax_scale, sl2, lse2, delta, sq_pad,
                       (unsigned long long*)((char*)a->workspace + pico_attn_bwd_split_workspace(a) - STAMP_BYTES),
                       q_front(a), use_kvp ? -1.0f / a->softmax_scale : LOG2E, use_kvp ? -INFINITY : INFINITY));
  const int nkb = (int)((a->seqlen_k + kv_block(a) - 1) / kv_block(a));
  const int hsplit = kv_hsplit(a);
  const BlkGroups kg = kv_groups(a, hsplit, kv_minb(a));
  const int64_t nblk = (int64_t)(kg.n ? kg.n : nkb) * a->batch * a->heads_kv * hsplit;
  if (nblk == 0) return 0;
  unsigned long long* stamps = (unsigned long long*)((char*)a->workspace + pico_attn_bwd_split_workspace(a) - STAMP_BYTES);
#ifndef PICO_SPLIT_D128_TU
  if (use_kvp && kvp_waves(a) == 8) {
    PICO_TRY(pico_launch(PICO_K_ATTN_BWD_KV, "attn_bwd_kv", attn_bwd_kvp_kernel<CAUSAL, 1, 8>, dim3((int)nblk),
                         dim3(8 * 64), 0, s, *a, a->softmax_scale, sl2, lse2, delta, sq_pad, hsplit, dkv_part, kg,
                         stamps));
  } else if (use_kvp) {
    PICO_TRY(pico_launch(PICO_K_ATTN_BWD_KV, "attn_bwd_kv", attn_bwd_kvp_kernel<CAUSAL, 2, 4>, dim3((int)nblk),
                         dim3(4 * 64), 0, s, *a, a->softmax_scale, sl2, lse2, delta, sq_pad, hsplit, dkv_part, kg,
                         stamps));
  } else
#else
  if (use_kvp) {
    PICO_TRY(pico_launch(PICO_K_ATTN_BWD_KV, "attn_bwd_kv", attn_bwd_kvp128_kernel<CAUSAL>, dim3((int)nblk),
                         dim3(4 * 64), 0, s, *a, a->softmax_scale, sl2, lse2, delta, sq_pad, hsplit, dkv_part, kg,
                         stamps));
  } else
#endif
  if constexpr (D == 128) {
    PICO_TRY(pico_launch(PICO_K_ATTN_BWD_KV, "attn_bwd_kv", attn_bwd_kv_kernel<D, CAUSAL, 1>, dim3((int)nblk),
                         dim3(KNW * 64), 0, s, *a, a->softmax_scale, sl2, lse2, delta, sq_pad, hsplit, dkv_part, stamps, kg));
  } else if constexpr (CAUSAL) {
    PICO_TRY(pico_launch(PICO_K_ATTN_BWD_KV, "attn_bwd_kv", attn_bwd_kv_kernel<D, CAUSAL, 3>, dim3((int)nblk),
                         dim3(KNW * 64), 0, s, *a, a->softmax_scale, sl2, lse2, delta, sq_pad, hsplit, dkv_part, stamps, kg));
  } else {
    PICO_TRY(pico_launch(PICO_K_ATTN_BWD_KV, "attn_bwd_kv", attn_bwd_kv_kernel<D, CAUSAL, 2>, dim3((int)nblk),
                         dim3(KNW * 64), 0, s, *a, a->softmax_scale, sl2, lse2, delta, sq_pad, hsplit, dkv_part, stamps, kg));
  }
  if (hsplit > 1) {
    const int kv_blocks = pico_cdiv(a->batch * a->seqlen_k * a->heads_kv * (D / 16), 256);
    PICO_TRY(pico_launch(PICO_K_ATTN_BWD_DKV, "attn_bwd_dkv", attn_bwd_dkv_kernel<D>, dim3(kv_blocks), dim3(256), 0, s, *a, dkv_part, hsplit));
  }
  return 0;
}

}  // namespace

// workspace of the split backward: [lse2 | delta] each [B*Hq][Sq_pad32] fp32 (+ fp32 dK/dV partials when
// a small grid splits key blocks): O(S), independent of the number of key blocks
#ifndef PICO_SPLIT_D128_TU
int64_t pico_attn_bwd_split_workspace(const pico_attn_args* a) {
  const int hs = kv_hsplit(a);
  const int64_t dkv = hs > 1 ? 2 * hs * a->batch * a->seqlen_k * a->heads_kv * a->head_dim : 0;
  return (2 * split_lsd_floats(a) + dkv) * 4 + STAMP_BYTES;
}
#endif

#ifndef PICO_SPLIT_D128_TU
int pico_attn_bwd_split_d128(const pico_attn_args* a, hipStream_t s);  // attn_bwd_split_d128.hip

int pico_attn_bwd_split(const pico_attn_args* a, hipStream_t s) {
  if (a->head_dim == 128) return pico_attn_bwd_split_d128(a, s);
  return a->causal ? launch_split<64, true>(a, s) : launch_split<64, false>(a, s);
}
#else
// head_dim 128: its own translation unit (its own per-file build flags, picotron_amd/build.py FILE_FLAGS)
int pico_attn_bwd_split_d128(const pico_attn_args* a, hipStream_t s) {
  return a->causal ? launch_split<128, true>(a, s) : launch_split<128, false>(a, s);
}
#endif
