// Flash-attention forward for head_dim 64 on gfx950: the two-half ping-pong form.
//
// Replaces flash_attn_func(q, k, v, causal) at D = 64 (ref picotron/model.py:32-36,153; SmolLM-1.7B's
// head_dim) and the ring block forward (ref picotron/context_parallel/context_parallel.py:112-128).
// Same contract as attn_fwd_kernel (attn_fwd.hip): bf16 in/out, fp32 online softmax, fp32 LSE, GQA,
// causal (Sq == Sk) or full, ragged S, PICO_ATTN_ROPE_Q_FWD, optional O^T output.
//
// Why a second D = 64 kernel. At D = 64 a 32-row x 64-key tile is 16 MFMAs (512 matrix cycles) against
// ~110 VALU instructions of softmax (32 exp at 8 issue cycles, 32 fma, 32 add, 16 max3, 16 cvt_pk: ~600
// issue cycles): the VALU, not the matrix pipe, bounds the loop. The 128-row kernel runs each wave as
// S MFMAs -> dependent softmax -> PV MFMAs, so a wave's MFMAs and its softmax never overlap and only the
// other waves of the SIMD can fill the gaps (PMC: SQ_WAIT_INST_ANY ~49 %, MFMA busy 15 %).
//
// Structure: one workgroup = 4 waves = 256 query rows of one (batch, q-head); each wave owns 64 rows as
// two 32-row halves A and B, offset by half a tile, so that one half's softmax VALU runs between the
// other half's MFMAs (cdna_hip_programming.md §Fused attention prefill, FA3-style intra-wave ping-pong):
//   segment A(t): VALU softmax of S_A(t) -> P_A(t)  | MFMA  S_B(t) = K(t) Q_B^T,  then O_A += V(t)^T P_A(t)
//   segment B(t): VALU softmax of S_B(t) -> P_B(t)  | MFMA  S_A(t+1) = K(t+1) Q_A^T,  then O_B += V(t)^T P_B(t)
// (P is consumed by the PV MFMAs 8 keys at a time as the exp VALU produces it, so it never needs registers
// beyond one operand.)
// The swapped product S^T = K Q^T keeps one query row per lane (lane-local softmax; P^T is directly the B
// operand of O^T += V^T P^T), as in attn_fwd.hip, whose LDS images (XOR-swizzled K, tr-read V) and
// LDS-DMA piece map this kernel reuses. 64-key tiles arrive by LDS-DMA into a 4-slot ring (prefetch
// distance 2 tiles), one barrier per tile, counted vmcnt waits. 64 KiB LDS and <= 256 VGPRs per wave:
// two workgroups per CU (two waves per SIMD).
// Causal grid: heaviest query blocks first, snaked per dispatch round (attn_fwd.hip PICO_FWD_SNAKE), so
// at S = 1024 every CU gets one heavy and one light block (16 + 4 or 12 + 8 tiles).
#include "attn_common.h"

#ifndef PICO_FWD64_THR
#define PICO_FWD64_THR 8  // lazy rescale threshold (log2 units), as PICO_FWD_RESCALE_THR
#endif
#ifndef PICO_FWD64_SCHED
#define PICO_FWD64_SCHED 2  // 2: hand-ordered MFMA slots; 0: compiler order
#endif

// PICO_FWD64_ABL: ablation builds for timing only (results are wrong): bit 1 no exp2 in the main block,
// 2 no operand LDS reads (registers stand in), 4 no tile wait / barrier in the loop, 8 no MFMAs in the main
// block, 32 no softmax segments at all, 64 no rescale check
#ifndef PICO_FWD64_ABL
#define PICO_FWD64_ABL 0
#endif
// PICO_FWD64_STAMP: diagnostic build -- every wave sums s_memtime cycles per phase (0 prologue, 1 mask + max
// phase, 2 main block, 3 tile wait + barrier, 4 DMA issue, 5 S-only segments, 6 epilogue, 7 total) and writes
// them to a.workspace[(blockIdx * 4 + wave) * 8 + phase] (uint64) when a.workspace is non-null
#ifndef PICO_FWD64_STAMP
#define PICO_FWD64_STAMP 0
#endif
#if PICO_FWD64_STAMP
#define FWD64_T(v) v = __builtin_amdgcn_s_memtime()
#define FWD64_ACC(bin, t0) do { const unsigned long long _t = __builtin_amdgcn_s_memtime(); ph[bin] += _t - (t0); (t0) = _t; } while (0)
#else
#define FWD64_T(v) do { } while (0)
#define FWD64_ACC(bin, t0) do { } while (0)
#endif

// PICO_FWD64_LSUM: the softmax row sums on the matrix pipe: one v_mfma_f32_16x16x32_bf16 per 16-key P^T
// fragment (the PV MFMA's own B operand) against a constant 0/1 A operand whose rows 0 and 1 select the
// k-slots of lanes 0-15 / 32-47 (query n) and 16-31 / 48-63 (query n + 16), so D[0][n] and D[1][n] are the
// two queries' partial sums (of the bf16-rounded P the PV product uses): 4 MFMAs of 16 cycles per
// segment instead of 36 VALU adds.
// PICO_FWD64_QSCALE: S arrives from the matrix pipe already in the exp2 argument's units, so the softmax
// needs no fma per score: q is prescaled by softmax_scale * log2(e) once (one extra bf16 rounding of q,
// relative 2^-9 per element, below the bf16 rounding of P itself), and the running max enters the S chain
// as one more MFMA, [ones | 0] x [-m | 0]^T (k-slot 0), so S' = scale log2e q.k - m. m is kept
// bf16-representable (it is only a stabiliser); a rescale subtracts the change from the pending S' too.
// Off: measured to break the LSE tolerance (C2: LSE max |err| 6.6e-3 vs 2e-3, O rel-L2 2.0e-3 -> 2.6e-3).
#ifndef PICO_FWD64_QSCALE
#define PICO_FWD64_QSCALE 0
#endif
#ifndef PICO_FWD64_LSUM
#define PICO_FWD64_LSUM 1
#endif
static_assert(!PICO_FWD64_QSCALE || (PICO_FWD64_LSUM && PICO_FWD64_SCHED == 2), "QSCALE keeps l in the row-sum MFMA accumulator and needs the hand-ordered block");
#ifndef PICO_FWD64_RD
#define PICO_FWD64_RD 3  // operand reads issued this many MFMA slots ahead of their consumer
#endif

namespace {

// Softmax VALU op k (0..111) of a segment's main block: 100 * type + 10 * chunk + index, type 0 fma, 1 exp2,
// 2 cvt_pk (index = pair), 3 row-sum add. Chunk order C0 C1 A0 C2 A1 C3 A2 A3 (C = 20 ops, A = 8 adds);
// inside C_c: f0..f3 e0..e3 f4..f7 v0 v1 e4..e7 v2 v3 (fma -> exp distance 4, exp -> cvt distance >= 2).
constexpr int fwd64_chunk_op(int j, int c) {
  constexpr int f = 0, e = 100, v = 200;
  const int seq[20] = {f + 0, f + 1, f + 2, f + 3, e + 0, e + 1, e + 2, e + 3, f + 4, f + 5,
                       f + 6, f + 7, v + 0, v + 1, e + 4, e + 5, e + 6, e + 7, v + 2, v + 3};
  return seq[j] + 10 * c;
}
// With S' prescaled (PICO_FWD64_QSCALE) a chunk is 8 exp2 then 4 cvt_pk (12 ops; C0 .. C3, 48 ops).
constexpr int fwd64_op_qs(int k) { return (k % 12 < 8 ? 100 + k % 12 : 200 + k % 12 - 8) + 10 * (k / 12); }
// With the row sums on the matrix pipe (PICO_FWD64_LSUM) the stream is C0 C1 C2 C3 only (80 ops).
constexpr int fwd64_op_lsum(int k) { return fwd64_chunk_op(k % 20, k / 20); }
constexpr int fwd64_op(int k) {
  // segments of the stream: {start, kind (0 = C, 1 = A), chunk}
  return k < 20   ? fwd64_chunk_op(k, 0)
         : k < 40 ? fwd64_chunk_op(k - 20, 1)
         : k < 48 ? 300 + 0 + (k - 40)
         : k < 68 ? fwd64_chunk_op(k - 48, 2)
         : k < 76 ? 300 + 10 + (k - 68)
         : k < 96 ? fwd64_chunk_op(k - 76, 3)
         : k < 104 ? 300 + 20 + (k - 96)
                   : 300 + 30 + (k - 104);
}

constexpr int BM = 256;  // query rows per workgroup (64 per wave)
constexpr int BN = 64;   // keys per tile
constexpr int D = 64;
constexpr int KS = 4;    // 16-wide k-steps of S^T over d
constexpr int DT = 2;    // 32-wide d tiles of O^T
constexpr int KIMG = BN * 32;        // one 16-wide K image [64 keys][16 d]
constexpr int VIMG = BN * 64;        // one 32-wide V image [64 keys][32 d]
constexpr int VBASE = BN * D * 2;    // V images follow the K images in a slot
constexpr int SLOT = 2 * BN * D * 2; // 16 KiB: K + V of one tile
constexpr int NBUF = 4;
constexpr int NIW = (2 * KS + 4 * DT) / 4;  // 1-KiB DMA pieces per wave per tile (4)

PICO_DEV float halves_max64(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
PICO_DEV float halves_sum64(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

template <bool CAUSAL>
__global__ __launch_bounds__(256, 2) __attribute__((amdgpu_waves_per_eu(2, 2)))
void attn_fwd64_kernel(const pico_attn_args a, float scale_log2, int round_len) {
  __shared__ __attribute__((aligned(16))) char smem[NBUF * SLOT];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
#if PICO_FWD64_STAMP
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tst, t_entry;
  FWD64_T(tst);
  t_entry = tst;
#endif

  // ---- block -> (query block, batch, head): heaviest first, snaked per round (see attn_fwd.hip) ----
  const int nmb = (int)((a.seqlen_q + BM - 1) / BM);
  const int nbh = (int)(a.batch * a.heads_q);
  int lin = blockIdx.x;
  if (CAUSAL) {
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
  const int ksd = (int)a.k_strides[1], vsd = (int)a.v_strides[1];

  const int q0 = mb * BM;
  const int qw = q0 + wave * 64;  // this wave's first row; half x owns rows qw + 32 x + (0..31)

  // ---- DMA tiles 0 .. NBUF-2 first (they are the critical path of the prologue) ----
  const int kend = CAUSAL ? min(Sk, q0 + BM) : Sk;
  const int ntiles = (kend + BN - 1) / BN;
  // piece j = wave + 4 i (attn_fwd.hip map): i < 2 are K pieces (j < 8): image j/2, rows 32 (j&1) + lane/2,
  // LDS chunk lane&1 holding source chunk (lane&1) ^ bit3(row); i >= 2 are V pieces: image i-2, rows
  // 16 wave + lane/4, 16-B part lane&3. Only the full-tile byte offsets stay in registers; the partial
  // last tile recomputes its clamped rows.
  auto piece_row = [&](int i) __attribute__((always_inline)) {
    return i < 2 ? 32 * (wave & 1) + (lane >> 1) : 16 * wave + (lane >> 2);
  };
  auto piece_col = [&](int i, int row) __attribute__((always_inline)) {
    return i < 2 ? 16 * ((wave + 4 * i) >> 1) + 8 * ((lane & 1) ^ ((row >> 3) & 1)) : 32 * (i - 2) + 8 * (lane & 3);
  };
  auto piece_dst = [&](int i) __attribute__((always_inline)) {
    return i < 2 ? (unsigned)(((wave + 4 * i) >> 1) * KIMG + (wave & 1) * 32 * 32)
                 : (unsigned)(VBASE + (i - 2) * VIMG + 16 * wave * 64);
  };
  unsigned full_off[NIW];  // byte offsets within a full tile
#pragma unroll
  for (int i = 0; i < NIW; ++i) {
    const int row = piece_row(i);
    full_off[i] = 2u * (unsigned)(row * (i < 2 ? ksd : vsd) + piece_col(i, row));
  }
  const unsigned smem_lds = lds_addr(smem);
  auto issue = [&](int tile) __attribute__((always_inline)) {
    const unsigned slot = smem_lds + (unsigned)(tile & (NBUF - 1)) * (unsigned)SLOT;
    const int base = tile * BN;
    const bf16_t* kt_ = kg + (int64_t)base * ksd;
    const bf16_t* vt_ = vg + (int64_t)base * vsd;
    if (base + BN <= Sk) {
#pragma unroll
      for (int i = 0; i < NIW; ++i) dma_piece(i < 2 ? kt_ : vt_, full_off[i], slot + piece_dst(i));
    } else {  // the last, partial tile clamps rows (finite values; the softmax masks keys >= Sk)
#pragma unroll
      for (int i = 0; i < NIW; ++i) {
        const int row = piece_row(i);
        const unsigned off = 2u * (unsigned)((min(base + row, Sk - 1) - base) * (i < 2 ? ksd : vsd) + piece_col(i, row));
        dma_piece(i < 2 ? kt_ : vt_, off, slot + piece_dst(i));
      }
    }
  };

  // ---- Q fragments (B operand of S^T = K Q^T): qf[x][ks] = Q[row][16 ks + 8 h .. +7] ----
  // Loaded by inline asm, like the DMA pieces, so that hipcc's own vmcnt bookkeeping (which cannot see
  // the asm DMA) does not drain the first tiles at the first use of q: the pieces are issued after these
  // loads, so the counted wait for tile 0 covers them, and the empty asm after it orders their uses.
  bf16x8 qf[2][KS];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const bf16_t* qp = qg + (int64_t)min(qw + 32 * x + r, Sq - 1) * a.q_strides[1] + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qf[x][ks]) : "v"(qp + 16 * ks) : "memory");
  }
  const bool rope_q = (a.flags & PICO_ATTN_ROPE_Q_FWD) != 0;
  u16x8 rc[2][KS / 2], rs[2][KS / 2];
  if (rope_q) {
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const int pos = min(qw + 32 * x + r, Sq - 1);
      const bf16_t* cp = (const bf16_t*)a.rope_cos + (int64_t)pos * a.rope_stride + 8 * h;
      const bf16_t* sp = (const bf16_t*)a.rope_sin + (int64_t)pos * a.rope_stride + 8 * h;
#pragma unroll
      for (int ks = 0; ks < KS / 2; ++ks) {
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(rc[x][ks]) : "v"(cp + 16 * ks) : "memory");
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(rs[x][ks]) : "v"(sp + 16 * ks) : "memory");
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NBUF - 1; ++t)
    if (t < ntiles) issue(t);
  // tile 0 (and, older, q and the tables) landed for this wave; then every wave's pieces
  wait_vmcnt(NIW * (min(NBUF - 1, ntiles) - 1));
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(qf[x][ks]));
  if (rope_q) {  // the rope kernel's arithmetic, bit for bit (attn_fwd.hip)
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int ks = 0; ks < KS / 2; ++ks) asm volatile("" : "+v"(rc[x][ks]), "+v"(rs[x][ks]));
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int ks = 0; ks < KS / 2; ++ks) {
        const u16x8 x1 = __builtin_bit_cast(u16x8, qf[x][ks]), x2 = __builtin_bit_cast(u16x8, qf[x][ks + KS / 2]);
        u16x8 o1, o2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xa = bf2f(x1[j]), xb = bf2f(x2[j]);
          const float cf = bf2f(rc[x][ks][j]), sf = bf2f(rs[x][ks][j]);
          o1[j] = f2bf(__fmul_rn(xa, cf) - __fmul_rn(xb, sf));
          o2[j] = f2bf(__fmul_rn(xb, cf) + __fmul_rn(xa, sf));
        }
        qf[x][ks] = __builtin_bit_cast(bf16x8, o1);
        qf[x][ks + KS / 2] = __builtin_bit_cast(bf16x8, o2);
      }
  }
  // With QSCALE the rotated rows leave now (the scaled copy replaces them in registers): 8 stores per lane,
  // unconditional (rows past Sq rewrite row Sq - 1 with its own value), counted in the loop's first waits.
  const int nq_st = (PICO_FWD64_QSCALE && rope_q) ? 2 * KS : 0;
  if (PICO_FWD64_QSCALE && rope_q) {
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const int row = min(qw + 32 * x + r, Sq - 1);
      bf16_t* rq = (bf16_t*)a.dq + b * a.dq_strides[0] + hq * a.dq_strides[2] + (int64_t)row * a.dq_strides[1] + 8 * h;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) *reinterpret_cast<u16x8*>(rq + 16 * ks) = __builtin_bit_cast(u16x8, qf[x][ks]);
    }
  }
  if (PICO_FWD64_QSCALE) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[x][ks][j] = (__bf16)((float)qf[x][ks][j] * scale_log2);
  }

  // ---- per-half causal / ragged limits (wave-uniform except lim_lane) ----
  int lim_first[2], last_t[2], lim_lane[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int row0 = qw + 32 * x;
    lim_first[x] = CAUSAL ? min(row0, Sk - 1) : Sk - 1;            // tiles ending <= this need no mask
    last_t[x] = (CAUSAL ? min(row0 + 31, Sk - 1) : Sk - 1) / BN;  // last tile with a visible key
    lim_lane[x] = CAUSAL ? min(row0 + r, Sk - 1) : Sk - 1;
  }

  // per-lane LDS read offsets (everything else is an immediate)
  const unsigned k_lane = r * 32 + 16 * (h ^ ((r >> 3) & 1));
  const unsigned v_lane = (4 * h + ((lane & 15) >> 2)) * 64 + 32 * ((lane >> 4) & 1) + 8 * (lane & 3);

  f32x16 O[2][DT], S[2][2];
  float m[2], l[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    m[x] = -INFINITY;
    l[x] = 0.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) O[x][dt] = (f32x16)0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) S[x][kt] = (f32x16)0.f;
  }

  // row-sum MFMA operand (PICO_FWD64_LSUM): lane l = 16 g + n holds A[n][8 g + j]; rows 0 / 1 are ones on the
  // k-slots of even / odd 16-lane groups
  bf16x8 ones_a;
  {
    const int n = lane & 15, g = lane >> 4;
    const bool one = (n == 0 && (g & 1) == 0) || (n == 1 && (g & 1) == 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) ones_a[j] = (__bf16)(one ? 1.f : 0.f);
  }
  f32x4 ls16[2] = {(f32x4)0.f, (f32x4)0.f};
  // PICO_FWD64_QSCALE: A = [1 | 0] (k-slot 0 of every key row: lanes h = 0, element 0) and per half
  // B = [-m | 0] (k-slot 0 of query r: lane r, element 0), so mfma(ones_k, bias[x]) = -m broadcast
  bf16x8 ones_k, bias[2];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ones_k[j] = (__bf16)(j == 0 && h == 0 ? 1.f : 0.f);
    bias[0][j] = bias[1][j] = (__bf16)0.f;
  }

  // ---- building blocks ----
  // V^T operand for keys 32 kt + 16 st .. +15 of the tile, d tile dt (two ds_read_b64_tr_b16)
  auto read_v = [&](const char* vb, int kt, int st, int dt) __attribute__((always_inline)) {
    return lds_read_tr_rows(vb + dt * VIMG + (32 * kt + 16 * st) * 64, 8 * 64);
  };
  auto kbase = [&](int tile) __attribute__((always_inline)) {
    return smem + (unsigned)(tile & (NBUF - 1)) * (unsigned)SLOT + k_lane;
  };
  auto vbase = [&](int tile) __attribute__((always_inline)) {
    return smem + (unsigned)(tile & (NBUF - 1)) * (unsigned)SLOT + v_lane + VBASE;
  };
  auto mask_s = [&](int x, int n0) __attribute__((always_inline)) {
    const int rel = lim_lane[x] - n0 - 4 * h;  // key n0 + c allowed iff c <= rel
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = 32 * kt + (i & 3) + 8 * (i >> 2);
        S[x][kt][i] = c <= rel ? S[x][kt][i] : -INFINITY;
      }
  };
  // scaled row max of the S a half will take next (computed when its S MFMAs finish, masked first when
  // the tile needs it), and the lazy rescale of O[x], l[x] against it (T13) at the start of its softmax
  float mt[2] = {-INFINITY, -INFINITY};
  auto tile_max = [&](int x) __attribute__((always_inline)) {
    float m0 = fmaxf(S[x][0][0], S[x][0][1]), m1 = fmaxf(S[x][1][0], S[x][1][1]);
#pragma unroll
    for (int i = 2; i < 16; i += 2) {
      m0 = __builtin_fmaxf(m0, __builtin_fmaxf(S[x][0][i], S[x][0][i + 1]));
      m1 = __builtin_fmaxf(m1, __builtin_fmaxf(S[x][1][i], S[x][1][i + 1]));
    }
    mt[x] = halves_max64(fmaxf(m0, m1)) * (PICO_FWD64_QSCALE ? 1.f : scale_log2);
  };
  auto rescale = [&](int x) __attribute__((always_inline)) {
#if PICO_FWD64_QSCALE
    // mt[x] is the excess of the pending S' over the current m (m = -inf: none yet, bias 0, mt = the max)
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(mt[x] > (float)PICO_FWD64_THR || m[x] == -INFINITY) != 0, 0)) {
      const bool first = m[x] == -INFINITY;
      const float m_new = (float)(__bf16)((first ? 0.f : m[x]) + fmaxf(mt[x], first ? mt[x] : 0.f));
      const float d = first ? m_new : m_new - m[x];  // exact: both bf16 values
      const float alpha = first ? 0.f : fast_exp2(-d);
      ls16[x][0] *= alpha;
      ls16[x][1] *= __shfl(alpha, (lane & 15) + 16);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) O[x][dt] *= alpha;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) S[x][kt] -= d;  // the pending S' was taken against the old m
      m[x] = m_new;
      bias[x][0] = (__bf16)(-m_new);
    }
#else
    if (__builtin_expect(__builtin_amdgcn_ballot_w64(mt[x] > m[x] + (float)PICO_FWD64_THR) != 0, 0)) {
      const float m_new = fmaxf(m[x], mt[x]);
      const float alpha = m[x] == -INFINITY ? 0.f : fast_exp2(m[x] - m_new);
      l[x] *= alpha;
      if (PICO_FWD64_LSUM) {  // lane n < 16 holds queries n (reg 0) and n + 16 (reg 1)
        ls16[x][0] *= alpha;
        ls16[x][1] *= __shfl(alpha, (lane & 15) + 16);
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) O[x][dt] *= alpha;
      m[x] = m_new;
    }
#endif
  };
  // P = exp2(scale log2e S - m) per 8-key step, packed to bf16 and fed at once to O^T += V^T P^T
  auto exp_pv = [&](int x, const char* vb) __attribute__((always_inline)) {
    const float neg_m = m[x] == -INFINITY ? 0.f : -m[x];
    float ls0 = 0.f, ls1 = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        float pv[8];
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
          pv[i] = fast_exp2(__builtin_fmaf(S[x][kt][8 * st + i], scale_log2, neg_m));
          pv[i + 1] = fast_exp2(__builtin_fmaf(S[x][kt][8 * st + i + 1], scale_log2, neg_m));
          ls0 += pv[i];
          ls1 += pv[i + 1];
        }
        const bf16x8 pf = pack_bf16x8(pv);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) O[x][dt] = mfma32(read_v(vb, kt, st, dt), pf, O[x][dt]);
      }
    l[x] += ls0 + ls1;
  };
  auto s_mfma = [&](int y, const char* kb) __attribute__((always_inline)) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      S[y][kt] = PICO_FWD64_QSCALE ? mfma32(ones_k, bias[y], (f32x16)0.f) : (f32x16)0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) S[y][kt] = mfma32(lds_read_b128(kb, ks * KIMG + kt * 32 * 32), qf[y][ks], S[y][kt]);
    }
  };

  // Steady-state body of a segment, hand-ordered (PICO_FWD64_SCHED == 2): 16 MFMA slots (S_Y: 8, then
  // O_X += V^T P_X: 8), each followed by 7 softmax VALU ops; sched_barrier(0) between slots keeps the order
  // (hipcc's waitcnt pass still counts each read's lgkmcnt). Operand reads run PICO_FWD64_RD slots ahead of
  // their MFMA (the first ones are issued before the max phase, whose VALU covers their latency).
  // VALU stream (fwd64_op): per 8-key chunk c = (kt, st) 8 fma, 8 exp2 and 4 cvt_pk interleaved (C_c, done
  // before its PV MFMAs at slots 8 + 2c), its 8 row-sum adds (A_c) one chunk later, so that at most two
  // chunks of exponentials are live: C0 C1 A0 C2 A1 C3 A2 A3.
  auto read = [&](auto u_tag, const char* kb, const char* vb, bf16x8 (&kf)[8], bf16x8 (&vf)[8])
      __attribute__((always_inline)) {
    constexpr int u = decltype(u_tag)::value;  // read unit u feeds MFMA slot u
    if constexpr ((PICO_FWD64_ABL & 2) != 0) {
      if constexpr (u < 8) kf[u] = qf[0][u & 3];
      else vf[u - 8] = qf[1][u & 3];
    } else if constexpr (u < 8) {
      kf[u] = lds_read_b128(kb, (u & 3) * KIMG + (u >> 2) * 32 * 32);  // K of S MFMA u: kt = u/4, ks = u%4
    } else {
      constexpr int pp = u - 8, c = pp >> 1, dt = pp & 1;
      vf[pp] = read_v(vb, c >> 1, c & 1, dt);
    }
  };
  auto main_block = [&](auto x_tag, auto fold_tag, const char* kb, const char* vb, bf16x8 (&kf)[8], bf16x8 (&vf)[8])
      __attribute__((always_inline)) {
    constexpr int X = decltype(x_tag)::value, Y = 1 - X;
    constexpr bool FOLD = decltype(fold_tag)::value;  // the row max of the new S_Y in the VALU stream
    float m0 = 0.f, m1 = 0.f;
    // max steps of S_Y: chain over kt = 0 in slots 6-7 (its last MFMA issued at slot 3), kt = 1 in slots
    // 10-11 (slot 7), the halves' swap and scaling in slot 13
    auto max_ops = [&](auto i_tag) __attribute__((always_inline)) {
      constexpr int i = decltype(i_tag)::value;
      if constexpr (FOLD && (i == 6 || i == 7 || i == 10 || i == 11)) {
        constexpr int kt = i >= 10 ? 1 : 0, j0 = (i & 1) * 4;
        float& mm = kt ? m1 : m0;
        static_for<4>([&](auto j_) {
          constexpr int j = j0 + decltype(j_)::value;
          if constexpr (j == 0) mm = fmaxf(S[Y][kt][0], S[Y][kt][1]);
          else mm = __builtin_fmaxf(mm, __builtin_fmaxf(S[Y][kt][2 * j], S[Y][kt][2 * j + 1]));
        });
      } else if constexpr (FOLD && i == 13) {
        mt[Y] = halves_max64(fmaxf(m0, m1)) * (PICO_FWD64_QSCALE ? 1.f : scale_log2);
      }
    };
    const float neg_m = m[X] == -INFINITY ? 0.f : -m[X];
    (void)neg_m;
    float ta[32], e[32], ls[4] = {0.f, 0.f, 0.f, 0.f};
    unsigned pk[16];
    auto valu = [&](auto k_tag) __attribute__((always_inline)) {
      constexpr int op = PICO_FWD64_QSCALE ? fwd64_op_qs(decltype(k_tag)::value)
                         : PICO_FWD64_LSUM ? fwd64_op_lsum(decltype(k_tag)::value) : fwd64_op(decltype(k_tag)::value);
      constexpr int ty = op / 100, c = (op / 10) % 10, j = op % 10, kt = c >> 1, st = c & 1;
      if constexpr (ty == 0) {
        ta[8 * c + j] = __builtin_fmaf(S[X][kt][8 * st + j], scale_log2, neg_m);
      } else if constexpr (ty == 1) {
        const float arg = PICO_FWD64_QSCALE ? S[X][kt][8 * st + j] : ta[8 * c + j];
        e[8 * c + j] = (PICO_FWD64_ABL & 1) ? arg : fast_exp2(arg);
      } else if constexpr (ty == 2) {
        typedef __attribute__((ext_vector_type(2))) float f32x2;
        typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
        pk[4 * c + j] = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){e[8 * c + 2 * j], e[8 * c + 2 * j + 1]}, bf16x2));
      } else {
        ls[j & 3] += e[8 * c + j];
      }
    };
    auto mfma_slot = [&](auto i_tag) __attribute__((always_inline)) {
      constexpr int i = decltype(i_tag)::value;
      if constexpr ((PICO_FWD64_ABL & 8) != 0) {
        if constexpr (i < 8) S[Y][i >> 2][i & 3] += __builtin_bit_cast(float, kf[i][0] == kf[i][1] ? 1u : 0u);
        else O[X][i & 1][0] += __builtin_bit_cast(float, pk[(i - 8) >> 1 << 2] ^ __builtin_bit_cast(unsigned, vf[i - 8][2] == vf[i-8][3] ? 1.f : 0.f));
      } else if constexpr (i < 8) {
        constexpr int kt = i >> 2, ks = i & 3;
        if constexpr (ks == 0 && PICO_FWD64_QSCALE) S[Y][kt] = mfma32(ones_k, bias[Y], (f32x16)0.f);
        S[Y][kt] = mfma32(kf[i], qf[Y][ks], (ks == 0 && !PICO_FWD64_QSCALE) ? (f32x16)0.f : S[Y][kt]);
      } else {
        constexpr int pp = i - 8, c = pp >> 1, dt = pp & 1;
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
        const u32x4 pw = {pk[4 * c], pk[4 * c + 1], pk[4 * c + 2], pk[4 * c + 3]};
        O[X][dt] = mfma32(vf[pp], __builtin_bit_cast(bf16x8, pw), O[X][dt]);
        if constexpr (PICO_FWD64_LSUM && dt == 1) ls16[X] = mfma16(ones_a, __builtin_bit_cast(bf16x8, pw), ls16[X]);
      }
    };
    // VALU ops per slot: 7 each (112 ops), or with the MFMA row sums 6 each in slots 0-12 and 2 in slot 13
    // (80 ops; chunk c's last cvt_pk lands by slot 7 + 2c, before its PV MFMAs at slot 8 + 2c)
    constexpr int NV = PICO_FWD64_QSCALE ? 48 : PICO_FWD64_LSUM ? 80 : 112;
    auto ops_begin = [](int i) constexpr {
      return PICO_FWD64_QSCALE ? (i * 4 < 48 ? i * 4 : 48) : PICO_FWD64_LSUM ? (i * 6 < 80 ? i * 6 : 80) : 7 * i;
    };
    __builtin_amdgcn_sched_barrier(0);
    static_for<16>([&](auto i_) {
      constexpr int i = decltype(i_)::value;
      mfma_slot(i_);
      constexpr int b0 = ops_begin(i), b1 = i == 15 ? NV : ops_begin(i + 1);
      static_for<b1 - b0>([&](auto j_) { valu(std::integral_constant<int, b0 + decltype(j_)::value>{}); });
      max_ops(i_);
      if constexpr (i + PICO_FWD64_RD < 16) read(std::integral_constant<int, i + PICO_FWD64_RD>{}, kb, vb, kf, vf);
      __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (!PICO_FWD64_LSUM) l[X] += (ls[0] + ls[1]) + (ls[2] + ls[3]);
  };

  // One segment: half X's softmax of tile ts and its O^T += V(ts)^T P^T (when do_soft), beside the other
  // half's S_Y = K(tk) Q_Y^T and its row max. S_Y is computed unconditionally (a slot of the ring always
  // holds finite or stale bytes; an S_Y that no softmax will read is harmless): conditional MFMA groups
  // would make the register allocator keep two copies of S_Y. A tile that needs a mask for half Y (causal
  // diagonal, ragged end) masks S_Y after the block and takes its max again (two such tiles per wave and
  // query block; a second instance of the block for them made the register allocator spill).
  auto segment = [&](auto x_tag, auto mask_tag, int ts, int tk) __attribute__((always_inline)) {
    constexpr int X = decltype(x_tag)::value, Y = 1 - X;
    if ((PICO_FWD64_ABL & 32) != 0) return;
    if ((PICO_FWD64_ABL & 64) == 0) rescale(X);
    FWD64_ACC(1, tst);
#if PICO_FWD64_SCHED == 2
    bf16x8 kf[8], vf[8];
    const char *kb = kbase(tk), *vb = vbase(ts);
    static_for<PICO_FWD64_RD>([&](auto u) { read(u, kb, vb, kf, vf); });
    main_block(x_tag, std::true_type{}, kb, vb, kf, vf);
#else
    s_mfma(Y, kbase(tk));
    exp_pv(X, vbase(ts));
    tile_max(Y);
#endif
    if constexpr (decltype(mask_tag)::value) {
      const int nk = tk * BN;
      if (nk + BN - 1 > lim_first[Y]) {  // the folded max saw unmasked scores: mask, then take the max again
        mask_s(Y, nk);
        tile_max(Y);
      }
    }
    FWD64_ACC(2, tst);
  };
  // tile t + 1 landed (this wave's pieces; tile t + 2's may stay in flight), then every wave's; every wave
  // is past segment B(t - 1), the last reader of tile t - 1's slot, which now takes tile t + 3
  auto barrier_dma = [&](int t) __attribute__((always_inline)) {
    if (!(PICO_FWD64_ABL & 4)) {
      // younger than tile t + 1: tile t + 2 (if issued) and, for t + 1 <= NBUF - 2, the prologue's q stores
      if (t + 1 < ntiles) wait_vmcnt((t + 2 < ntiles ? NIW : 0) + (t + 1 <= NBUF - 2 ? nq_st : 0));
      lds_barrier();
    }
    FWD64_ACC(3, tst);
    if (t + NBUF - 1 < ntiles) issue(t + NBUF - 1);
    FWD64_ACC(4, tst);
  };

  // ---- prologue: S_A(0) ----
  lds_barrier();
  FWD64_ACC(0, tst);
  s_mfma(0, kbase(0));
  if (BN - 1 > lim_first[0]) mask_s(0, 0);
  tile_max(0);
  FWD64_ACC(5, tst);

  // ---- main loop: segment A(t) | barrier + DMA | segment B(t) ----
  // Both halves of a wave see their last key in the same tile td (qw is a multiple of 64); S tiles < td need
  // no mask, so iterations t < td - 1 run the mask-free segments, t = td - 1, td the masking ones (S_A(td),
  // S_B(td); the S_A(td + 1) of the last one is never read), and the rest of the workgroup's tiles only keep
  // this wave's share of the barriers and the DMA. No per-segment "is this half active" branch: the
  // conditional O / S updates it needed made hipcc copy the accumulators around every segment.
  const int td = last_t[0];
  int t = 0;
  for (; t < td - 1; ++t) {
    segment(std::integral_constant<int, 0>{}, std::false_type{}, t, t);
    barrier_dma(t);
    segment(std::integral_constant<int, 1>{}, std::false_type{}, t, t + 1);
  }
  for (; t <= td; ++t) {
    segment(std::integral_constant<int, 0>{}, std::true_type{}, t, t);
    barrier_dma(t);
    segment(std::integral_constant<int, 1>{}, std::true_type{}, t, t + 1);
  }
  for (; t < ntiles; ++t) barrier_dma(t);

  FWD64_ACC(5, tst);
  // ---- epilogue: O = O^T / l, LSE = (m + log2 l) ln 2; rotated q rows; O^T through LDS ----
  float inv[2], ltot[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    if (PICO_FWD64_LSUM) {  // query r's sum: lane r & 15, reg r >> 4 of the row-sum accumulator
      const float l0 = __shfl(ls16[x][0], r & 15), l1 = __shfl(ls16[x][1], r & 15);
      ltot[x] = r < 16 ? l0 : l1;
    } else {
      ltot[x] = halves_sum64(l[x]);
    }
    inv[x] = ltot[x] > 0.f ? 1.f / ltot[x] : 0.f;
  }
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    const int my_q = qw + 32 * x + r;
    const bool row_ok = my_q < Sq;
    bf16_t* op = (bf16_t*)a.o + b * a.o_strides[0] + hq * a.o_strides[2] + (int64_t)min(my_q, Sq - 1) * a.o_strides[1];
    store_row_bf16_x16<DT>(op, h, row_ok, [&](int dt, int i) { return O[x][dt][i] * inv[x]; });
    if (!PICO_FWD64_QSCALE && rope_q && row_ok) {
      bf16_t* rq = (bf16_t*)a.dq + b * a.dq_strides[0] + hq * a.dq_strides[2] + (int64_t)my_q * a.dq_strides[1] + 8 * h;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) *reinterpret_cast<u16x8*>(rq + 16 * ks) = __builtin_bit_cast(u16x8, qf[x][ks]);
    }
    if (h == 0 && row_ok) {
      const float lse = ltot[x] > 0.f ? (m[x] + __log2f(ltot[x])) * LN2 : -INFINITY;
      a.lse[((int64_t)b * a.heads_q + hq) * Sq + my_q] = lse;
    }
  }
  if (a.o_t) {  // uniform: O^T [Hq*D][tokens], staged transposed in the idle ring, 16-byte token runs
    constexpr int TP = BM + 8;
    static_assert(D * TP * 2 <= NBUF * SLOT, "O^T staging tile must fit the ring");
    unsigned short* tt = reinterpret_cast<unsigned short*>(smem);
    __syncthreads();
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int d = 32 * dt + 8 * (i >> 2) + 4 * h + (i & 3);
          tt[d * TP + 64 * wave + 32 * x + r] = f2bf(O[x][dt][i] * inv[x]);
        }
    __syncthreads();
    bf16_t* otb = (bf16_t*)a.o_t + (int64_t)hq * D * a.o_t_ld + (int64_t)b * Sq;
    const bool vec = ((a.o_t_ld | (int64_t)Sq | (int64_t)(uintptr_t)a.o_t) & 7) == 0;
    for (int seg = threadIdx.x; seg < D * BM / 8; seg += 256) {
      const int d = seg / (BM / 8), t8 = seg % (BM / 8);
      const int tok0 = q0 + 8 * t8;
      if (tok0 >= Sq) continue;
      bf16_t* dst = otb + (int64_t)d * a.o_t_ld + tok0;
      const unsigned short* src = tt + d * TP + 8 * t8;
      if (vec && tok0 + 8 <= Sq) {
        *reinterpret_cast<u16x8*>(dst) = *reinterpret_cast<const u16x8*>(src);
      } else {
        for (int j = 0; j < 8 && tok0 + j < Sq; ++j) dst[j] = src[j];
      }
    }
  }
#if PICO_FWD64_STAMP
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  FWD64_ACC(6, tst);
  ph[7] = tst - t_entry;
  if (a.workspace && lane < 8) {
    unsigned long long v = ph[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) v = lane == i ? ph[i] : v;
    ((unsigned long long*)a.workspace)[((int64_t)blockIdx.x * 4 + wave) * 8 + lane] = v;
  }
#endif
}

}  // namespace

// D = 64 forward, ping-pong form: whether this kernel takes the call (32-bit per-tile DMA offsets), and
// the launch.
bool pico_attn_fwd64_pp_ok(const pico_attn_args* a) {
  if (a->head_dim != 64) return false;
  if (a->k_strides[1] * 2 * BN >= (1ll << 31) || a->v_strides[1] * 2 * BN >= (1ll << 31)) return false;
  return (a->seqlen_q + BM - 1) / BM * a->batch * a->heads_q < (1ll << 31);
}

int pico_attn_fwd64_pp(const pico_attn_args* a, hipStream_t s) {
  const int nmb = (int)((a->seqlen_q + BM - 1) / BM);
  const int64_t nblk = (int64_t)nmb * a->batch * a->heads_q;
  const float sl2 = a->softmax_scale * LOG2E;
  const int rl = pico_num_cus() / 8 * 8 > 0 ? pico_num_cus() / 8 * 8 : 8;
  if (a->causal) {
    PICO_TRY(pico_launch(PICO_K_ATTN_FWD, "attn_fwd", attn_fwd64_kernel<true>, dim3((int)nblk), dim3(256), 0, s, *a, sl2, rl));
  } else {
    PICO_TRY(pico_launch(PICO_K_ATTN_FWD, "attn_fwd", attn_fwd64_kernel<false>, dim3((int)nblk), dim3(256), 0, s, *a, sl2, rl));
  }
  return 0;
}
