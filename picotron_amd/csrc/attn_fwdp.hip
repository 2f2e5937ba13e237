// Flash-attention forward for gfx950, persistent two-half form (round 6): one wave per SIMD, 64 query rows per wave.
//
// Replaces flash_attn_func(q, k, v, causal) (ref picotron/model.py:32-36,153; eager oracle
// F.scaled_dot_product_attention :156) and the ring block forward (ref picotron/context_parallel/context_parallel.py:
// 112-128) for the shapes the model runs: seqlen_q == seqlen_k (causal) or any lengths (non-causal), both multiples
// of 64, head_dim 64 or 128. attn_fwd.hip's 32-row kernel serves every other shape.
//
// Why this form (cdna_hip_programming.md "4-wave, one-wave-per-SIMD, persistent structure"):
// the 32-row kernel keeps four waves per SIMD, each one dependency chain per tile (S MFMAs -> softmax VALU -> PV
// MFMAs), and the SIMD's issue arbitration between them left the MFMA pipe 0.22 busy at C2. Here each wave owns
// 64 query rows as two 32-row halves A and B whose chains are offset by half a tile, so every MFMA phase of one
// half carries the other half's softmax VALU:
//     Ph1: S_A(t)       | softmax tail of B(t-1)  (exp of keys 32-63, pack P)
//     Ph2: PV_B(t-1)    | softmax head of A(t)    (row max, rescale vote, exp of keys 0-31)
//     Ph3: S_B(t)       | softmax tail of A(t)    + V(t) transposed reads
//     --- wait for tile t+1, workgroup barrier ---
//     Ph4: PV_A(t)      | softmax head of B(t)    + K(t+1) reads + LDS-DMA of tile t+NBUF-1
// One workgroup = 4 waves = a 256-row item of one (batch, q-head); K/V 64-key tiles stream through an NBUF-slot
// LDS ring (LDS-DMA, XOR-swizzled images as attn_fwd.hip), one barrier per tile. Workgroups are persistent over two
// items of one head for causal balance: query blocks J and nJ-1-J (4J+4 + 4(nJ-1-J)+4 tiles: equal for every
// workgroup), K/V streamed continuously across the seam.
// Causal diagonal: wave w's rows 64w..64w+63 of block J meet keys 64(4J+w).. on tile 4J+w exactly (Sq == Sk, 64 | S),
// so the mask of that tile is a fixed 32x32 pattern entering as the S MFMA chain's initial accumulator (0 / -inf),
// and the tiles after it are idle for the wave (it keeps its share of the DMA and the barriers).
#include <type_traits>

#include "attn_common.h"

#ifndef PICO_FWDP_RESCALE_THR
#define PICO_FWDP_RESCALE_THR 8
#endif
// PICO_FWDP_STAMP: diagnostic build (results unchanged, timing perturbed ~10 %) — every wave accumulates s_memtime
// deltas per phase into 16 x 8 B at a.workspace[(block * 4 + wave) * 16] (scripts/fwdp_stamps.py): 0 Ph1, 1 Ph2,
// 2 Ph3, 3 DMA wait, 4 barrier, 5 DMA issue, 6 Ph4, 7 idle tiles, 8 item prologue, 9 epilogue, 10 B tail,
// 11 active tiles, 12 wave lifetime, 13 s_memrealtime at start, 14 at end
#ifndef PICO_FWDP_STAMP
#define PICO_FWDP_STAMP 0
#endif
#if PICO_FWDP_STAMP
#define FP_ST(i)                                              \
  {                                                           \
    __builtin_amdgcn_sched_barrier(0);                        \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    ph[i] += t_ - tlast;                                      \
    tlast = t_;                                               \
    __builtin_amdgcn_sched_barrier(0);                        \
  }
#else
#define FP_ST(i)
#endif

namespace {

constexpr int PB = 256;  // query rows per item (4 waves x 64)
constexpr int PN = 64;   // keys per tile

template <int D>
struct PCfg {
  static constexpr int KS = D / 16, DT = D / 32;
  static constexpr int KIMG = PN * 32;         // one 16-wide K image [64 keys][16 d]
  static constexpr int VIMG = PN * 64;         // one 32-wide V image [64 keys][32 d]
  static constexpr int SLOT = 2 * PN * D * 2;  // K + V of one tile
  static constexpr int NBUF = D == 64 ? 4 : 3;
  static constexpr int NI = 2 * KS + 4 * DT;   // 1-KiB DMA pieces per tile
  static constexpr int NIW = NI / 4;           // ... per wave
  static constexpr int RING = NBUF * SLOT;
  static constexpr int TP = 64 + 8;            // pitch (elements) of a wave's O^T staging tile [64 d][64 rows]
  static constexpr int OTW = 64 * TP * 2;      // bytes per wave
  static constexpr int LDS = RING + 4 * OTW;
};

PICO_DEV float hmax(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
PICO_DEV float hsum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Keep a value's computation above this point: an empty volatile asm that reads and redefines it (machine sinking
// would otherwise move a phase's softmax VALU down to its consumer, past the tile's barrier, and serialise it there)
template <typename T>
PICO_DEV void pin(T& x) {
  asm volatile("" : "+v"(x));
}

template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void attn_fwdp_kernel(const pico_attn_args a, float sl2, int nJ, int pairs) {
  using C = PCfg<D>;
  constexpr int KS = C::KS, DT = C::DT;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
#if PICO_FWDP_STAMP
  unsigned long long ph[16] = {0};
  ph[13] = __builtin_amdgcn_s_memrealtime();
  unsigned long long tlast = __builtin_amdgcn_s_memtime();
  const unsigned long long tstart = tlast;
#endif

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const int Sq = (int)a.seqlen_q, Sk = (int)a.seqlen_k;
  const int nbh = (int)(a.batch * a.heads_q);
  const int bh = blockIdx.x % nbh, p = blockIdx.x / nbh;
  const int b = bh / (int)a.heads_q, hq = bh % (int)a.heads_q;
  const int hk = hq / (int)(a.heads_q / a.heads_kv);
  // items of this workgroup: pairs -> blocks nJ-1-p and p (one if they coincide); else block nJ-1-p (causal, LPT
  // order) or p
  int Jit[2], nit = 1;
  if (pairs) {
    Jit[0] = nJ - 1 - p;
    Jit[1] = p;
    nit = Jit[0] == Jit[1] ? 1 : 2;
  } else {
    Jit[0] = CAUSAL ? nJ - 1 - p : p;
    Jit[1] = Jit[0];
  }
  const int nkt = Sk / PN;
  auto item_tiles = [&](int J) { return CAUSAL ? min(nkt, (J * PB + PB) / PN) : nkt; };
  const int nt0 = item_tiles(Jit[0]);
  const int gtot = nt0 + (nit > 1 ? item_tiles(Jit[1]) : 0);

  const bf16_t* qg = (const bf16_t*)a.q + b * a.q_strides[0] + hq * a.q_strides[2];
  const char* const kbase = (const char*)((const bf16_t*)a.k + b * a.k_strides[0] + hk * a.k_strides[2]);
  const char* const vbase = (const char*)((const bf16_t*)a.v + b * a.v_strides[0] + hk * a.v_strides[2]);
  const int64_t ksd = a.k_strides[1], vsd = a.v_strides[1];
  const int64_t kst = (int64_t)PN * ksd * 2, vst = (int64_t)PN * vsd * 2;  // bytes per tile

  // ---- LDS-DMA: piece j = wave + 4 i of a tile (K pieces j < 2 KS, then V), as attn_fwd.hip ----
  unsigned src_off[C::NIW], dst_off[C::NIW];
#pragma unroll
  for (int i = 0; i < C::NIW; ++i) {
    const int j = wave + 4 * i;
    if (j < 2 * KS) {
      const int ks = j >> 1, row = 32 * (j & 1) + (lane >> 1);
      src_off[i] = (unsigned)(row * ksd + 16 * ks + 8 * ((lane & 1) ^ ((row >> 3) & 1))) * 2u;
      dst_off[i] = ks * C::KIMG + 32 * (j & 1) * 32;
    } else {
      const int jv = j - 2 * KS, dt = jv >> 2, row = 16 * (jv & 3) + (lane >> 2);
      src_off[i] = (unsigned)(row * vsd + 32 * dt + 8 * (lane & 3)) * 2u;
      dst_off[i] = PN * D * 2 + dt * C::VIMG + 16 * (jv & 3) * 64;
    }
  }
  const unsigned ring0 = (unsigned)__builtin_amdgcn_readfirstlane((int)lds_addr(smem));
  // global tile g of the workgroup's stream -> (item tile) -> DMA into slot g % NBUF
  auto issue = [&](int g) __attribute__((always_inline)) {
    const int tl = g < nt0 ? g : g - nt0;
    const unsigned sl = ring0 + (unsigned)(g % C::NBUF) * (unsigned)C::SLOT;
#pragma unroll
    for (int i = 0; i < C::NIW; ++i) {
      const bool isk = wave + 4 * i < 2 * KS;  // uniform per (wave, i)
      dma_piece(isk ? kbase + tl * kst : vbase + tl * vst, src_off[i], sl + dst_off[i]);
    }
  };
  // wait until this wave's DMA pieces of tile g landed. Steady state: the pieces of the NBUF - 3 younger tiles stay in
  // flight (a constant count); near the end of the stream, or with stores issued after the pieces (an item's
  // epilogue), more than needed is waited for — never less (vmcnt counts every vector-memory op in issue order)
  int g_issued = 0;
  auto wait_tile = [&](int g) __attribute__((always_inline)) {
    if (C::NBUF > 3 && g_issued - 1 - g == C::NBUF - 3) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((C::NBUF - 3) * C::NIW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };
  for (; g_issued < C::NBUF - 1 && g_issued < gtot; ++g_issued) issue(g_issued);

  // per-lane LDS read offsets
  const unsigned k_lane = r * 32 + 16 * (h ^ ((r >> 3) & 1));
  const unsigned v_lane = (4 * h + ((lane & 15) >> 2)) * 64 + 32 * ((lane >> 4) & 1) + 8 * (lane & 3);
  const unsigned smem_lds = lds_addr(smem);

  // diagonal-tile mask pattern of a 32x32 block (key index of register i vs query r): 0 or -inf (built on the tile)
  auto mask_pattern = [&]() __attribute__((always_inline)) {
    f32x16 mp;
#pragma unroll
    for (int i = 0; i < 16; ++i) mp[i] = ((i & 3) + 8 * (i >> 2) + 4 * h > r) ? -INFINITY : 0.f;
    return mp;
  };

  const float inv_sl2 = 1.f / sl2;
  const bool rope_q = (a.flags & PICO_ATTN_ROPE_Q_FWD) != 0;

  int g = 0;  // global tile index of the stream
#pragma clang loop unroll(disable)
  for (int it = 0; it < nit; ++it) {
    const int J = Jit[it];
    const int q0 = J * PB;
    const int ntiles = item_tiles(J);
    const int wrow = q0 + 64 * wave;  // this wave's first row
    const bool wvalid = wrow < Sq;
    const int last_w = !wvalid ? -1 : (CAUSAL ? wrow / PN : ntiles - 1);
    FP_ST(9);  // (the previous item's epilogue / the kernel start)

    // ---- Q fragments of halves A (X = 0) and B (X = 1): B operand of S^T = K Q^T ----
    bf16x8 qf[2][KS];
    u16x8 rc[2][KS / 2], rs[2][KS / 2];
#pragma unroll
    for (int X = 0; X < 2; ++X) {
      const int row = min(wrow + 32 * X + r, Sq - 1);
      const bf16_t* qp = qg + (int64_t)row * a.q_strides[1] + 8 * h;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) qf[X][ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u16x8*>(qp + 16 * ks));
      if (rope_q) {
        const bf16_t* cp = (const bf16_t*)a.rope_cos + (int64_t)row * a.rope_stride + 8 * h;
        const bf16_t* sp = (const bf16_t*)a.rope_sin + (int64_t)row * a.rope_stride + 8 * h;
#pragma unroll
        for (int ks = 0; ks < KS / 2; ++ks) {
          rc[X][ks] = *reinterpret_cast<const u16x8*>(cp + 16 * ks);
          rs[X][ks] = *reinterpret_cast<const u16x8*>(sp + 16 * ks);
        }
      }
    }
    // Q (and every tile already issued) landed: the builtin form, so the compiler's own wait insertion knows the Q
    // loads are complete and puts no vmcnt of its own into the tile loop (vmcnt(0) expcnt(7) lgkmcnt(15))
    __builtin_amdgcn_s_waitcnt(0x0F70);
    if (rope_q) {  // rotate in registers (pico_rope's fp32 arithmetic, one rounding)
#pragma unroll
      for (int X = 0; X < 2; ++X)
#pragma unroll
        for (int ks = 0; ks < KS / 2; ++ks) {
          const u16x8 x1 = __builtin_bit_cast(u16x8, qf[X][ks]), x2 = __builtin_bit_cast(u16x8, qf[X][ks + KS / 2]);
          u16x8 o1, o2;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float xa = bf2f(x1[j]), xb = bf2f(x2[j]);
            const float cf = bf2f(rc[X][ks][j]), sf = bf2f(rs[X][ks][j]);
            o1[j] = f2bf(__fmul_rn(xa, cf) - __fmul_rn(xb, sf));
            o2[j] = f2bf(__fmul_rn(xb, cf) + __fmul_rn(xa, sf));
          }
          qf[X][ks] = __builtin_bit_cast(bf16x8, o1);
          qf[X][ks + KS / 2] = __builtin_bit_cast(bf16x8, o2);
        }
    }
    __builtin_amdgcn_s_barrier();  // every wave's pieces of the first tiles visible

    f32x16 o[2][DT];
#pragma unroll
    for (int X = 0; X < 2; ++X)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[X][dt] = (f32x16)0.f;
    float m[2] = {-INFINITY, -INFINITY}, negm[2] = {0.f, 0.f}, thr[2] = {-INFINITY, -INFINITY};
    float l[2] = {0.f, 0.f};
    f32x16 s[2][2];      // S^T accumulators [half][32-key block]
    bf16x8 pf[2][2][2];  // packed P^T [half][32-key block][16-key k-step]
    bf16x8 kf[2][KS];    // K fragments of the current tile [32-key block][k-step]
    bf16x8 vf[2][2][DT]; // V^T fragments [32-key block][16-key k-step][32-d tile]

    auto read_k = [&](int gg) __attribute__((always_inline)) {
      const char* kb = smem + ((unsigned)(gg % C::NBUF) * (unsigned)C::SLOT + k_lane);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) kf[kt][ks] = lds_read_b128(kb, ks * C::KIMG + kt * 32 * 32);
    };
    auto read_v = [&](int gg) __attribute__((always_inline)) {
      const unsigned va = smem_lds + (unsigned)(gg % C::NBUF) * (unsigned)C::SLOT + v_lane;
      static_for<2>([&](auto kt_) {
        constexpr int KT = decltype(kt_)::value;
        static_for<2>([&](auto st_) {
          constexpr int ST = decltype(st_)::value;
          static_for<DT>([&](auto dt_) {
            constexpr int DTI = decltype(dt_)::value;
            vf[KT][ST][DTI] = tr_operand_imm<PN * D * 2 + DTI * C::VIMG + (32 * KT + 16 * ST) * 64, 8 * 64>(va);
          });
        });
      });
    };
    // S^T of half X (one 32-key block kt): 4 (D 64) / 8 MFMAs; MASKK: the chain starts from cinit
    auto s_mfma = [&](int X, int kt, const f32x16& cinit) __attribute__((always_inline)) {
      s[X][kt] = mfma32(kf[kt][0], qf[X][0], cinit);
#pragma unroll
      for (int ks = 1; ks < KS; ++ks) s[X][kt] = mfma32(kf[kt][ks], qf[X][ks], s[X][kt]);
    };
    // softmax head of half X: row max over both key blocks, rescale vote (rare branch), P of key block 0
    auto sm_head = [&](int X) __attribute__((always_inline)) {
      float m0 = fmaxf(s[X][0][0], s[X][0][1]), m1 = fmaxf(s[X][1][0], s[X][1][1]);
#pragma unroll
      for (int i = 2; i < 16; ++i) {
        m0 = fmaxf(m0, s[X][0][i]);
        m1 = fmaxf(m1, s[X][1][i]);
      }
      const float mx = fmaxf(m0, m1);
      if (__builtin_amdgcn_ballot_w64(mx > thr[X])) {
        const float mn = fmaxf(m[X], hmax(mx) * sl2);
        const float alpha = m[X] == -INFINITY ? 0.f : fast_exp2(m[X] - mn);
        l[X] *= alpha;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[X][dt] *= alpha;
        m[X] = mn;
        negm[X] = mn == -INFINITY ? 0.f : -mn;
        thr[X] = (mn + (float)PICO_FWDP_RESCALE_THR) * inv_sl2;
      }
      float l0 = 0.f, l1 = 0.f;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const float p0 = fast_exp2(__builtin_fmaf(s[X][0][i], sl2, negm[X]));
        const float p1 = fast_exp2(__builtin_fmaf(s[X][0][i + 1], sl2, negm[X]));
        s[X][0][i] = p0;
        s[X][0][i + 1] = p1;
        l0 += p0;
        l1 += p1;
      }
      l[X] += l0 + l1;
    };
    // softmax tail of half X: P of key block 1, pack both blocks to bf16 (B operands of PV)
    auto sm_tail = [&](int X) __attribute__((always_inline)) {
      float l0 = 0.f, l1 = 0.f;
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const float p0 = fast_exp2(__builtin_fmaf(s[X][1][i], sl2, negm[X]));
        const float p1 = fast_exp2(__builtin_fmaf(s[X][1][i + 1], sl2, negm[X]));
        s[X][1][i] = p0;
        s[X][1][i + 1] = p1;
        l0 += p0;
        l1 += p1;
      }
      l[X] += l0 + l1;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        float pv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) pv[j] = s[X][kt][j];
        pf[X][kt][0] = pack_bf16x8(pv);
        pf[X][kt][1] = pack_bf16x8(pv + 8);
      }
    };
    auto pin_p = [&](int X) __attribute__((always_inline)) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int st = 0; st < 2; ++st) pin(pf[X][kt][st]);
      pin(l[X]);
    };
    auto pv_mfma = [&](int X) __attribute__((always_inline)) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[X][dt] = mfma32(vf[kt][st][dt], pf[X][kt][st], o[X][dt]);
    };
    // the wait + barrier of tile gg (the next tile landed everywhere) and the ring's next DMA
    auto sync_next = [&](int gg) __attribute__((always_inline)) {
      wait_tile(gg + 1 < gtot ? gg + 1 : gtot - 1);
      FP_ST(3);
      __builtin_amdgcn_s_barrier();
      FP_ST(4);
      if (g_issued < gtot && g_issued <= gg + C::NBUF - 1) {
        issue(g_issued);
        ++g_issued;
      }
      FP_ST(5);
    };

    // one tile of the wave's stream; FIRST: no B(t-1) work; MASKT: the diagonal tile (causal)
    auto body = [&](int gg, auto first_tag, auto mask_tag) __attribute__((always_inline)) {
      constexpr bool FIRST = decltype(first_tag)::value, MASKT = decltype(mask_tag)::value;
      const f32x16 mpat = MASKT ? mask_pattern() : (f32x16)0.f;
      // Ph1: S_A(t) | tail of B(t-1)
      s_mfma(0, 0, MASKT ? mpat : (f32x16)0.f);
      s_mfma(0, 1, MASKT ? (f32x16)(-INFINITY) : (f32x16)0.f);
      if constexpr (!FIRST) {
        sm_tail(1);
        pin_p(1);
      }
      FP_ST(0);
      // Ph2: PV_B(t-1) | head of A(t)
      if constexpr (!FIRST) pv_mfma(1);
      sm_head(0);
      pin(s[0][0]);
      FP_ST(1);
      // Ph3: S_B(t) | tail of A(t) + V(t) reads
      s_mfma(1, 0, (f32x16)0.f);
      s_mfma(1, 1, MASKT ? mpat : (f32x16)0.f);
      read_v(gg);
      sm_tail(0);
      pin_p(0);
      lds_wait_all();  // V(t) (inline-asm reads: the compiler does not count them) before PV_A(t) / PV_B(t)
      FP_ST(2);
      sync_next(gg);
      // Ph4: PV_A(t) | head of B(t) + K(t+1) reads
      pv_mfma(0);
      sm_head(1);
      pin(s[1][0]);
      read_k(gg + 1);
      FP_ST(6);
#if PICO_FWDP_STAMP
      ph[11] += 1;
#endif
    };
    // the last active tile's B tail (no next tile of this wave to carry it)
    auto btail = [&]() __attribute__((always_inline)) {
      sm_tail(1);
      pv_mfma(1);
      FP_ST(10);
    };
    auto idle = [&](int gg) __attribute__((always_inline)) {
      sync_next(gg);
      FP_ST(7);
    };

    read_k(g);
    FP_ST(8);
    const std::false_type F{};
    const std::true_type T{};
    int t = 0;
    if (last_w >= 0) {
      if (last_w == 0) {
        if constexpr (CAUSAL) body(g, T, T);
        else body(g, T, F);
        btail();
      } else {
        body(g, T, F);
      }
      t = 1;
#pragma clang loop unroll(disable)
      for (; t < last_w; ++t) body(g + t, F, F);
      if (last_w > 0) {
        if constexpr (CAUSAL) body(g + last_w, F, T);
        else body(g + last_w, F, F);
        btail();
        t = last_w + 1;
      }
    }
#pragma clang loop unroll(disable)
    for (; t < ntiles; ++t) idle(g + t);
    g += ntiles;

    // ---- epilogue of the item: O = O^T / l, LSE = (m + log2 l) ln 2; O^T through this wave's LDS staging ----
    if (wvalid) {
      float inv[2], ltot[2];
#pragma unroll
      for (int X = 0; X < 2; ++X) {
        ltot[X] = hsum(l[X]);
        inv[X] = ltot[X] > 0.f ? 1.f / ltot[X] : 0.f;
        const int row = wrow + 32 * X + r;
        const bool ok = row < Sq;
        bf16_t* op = (bf16_t*)a.o + b * a.o_strides[0] + hq * a.o_strides[2] + (int64_t)min(row, Sq - 1) * a.o_strides[1];
        const float iv = inv[X];
        store_row_bf16_x16<DT>(op, h, ok, [&](int dt, int i) { return o[X][dt][i] * iv; });
        if (rope_q && ok) {
          bf16_t* rq = (bf16_t*)a.dq + b * a.dq_strides[0] + hq * a.dq_strides[2] + (int64_t)row * a.dq_strides[1] + 8 * h;
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) *reinterpret_cast<u16x8*>(rq + 16 * ks) = __builtin_bit_cast(u16x8, qf[X][ks]);
        }
        if (h == 0 && ok) {
          a.lse[((int64_t)b * a.heads_q + hq) * Sq + row] = ltot[X] > 0.f ? (m[X] + __log2f(ltot[X])) * LN2 : -INFINITY;
        }
      }
      if (a.o_t) {  // O^T [Hq*D][tokens]: per 64-d pass, [64 d][64 rows] staged, 16-byte row segments stored
        unsigned short* tt = reinterpret_cast<unsigned short*>(smem + C::RING + wave * C::OTW);
        bf16_t* otb = (bf16_t*)a.o_t + (int64_t)hq * D * a.o_t_ld + (int64_t)b * Sq + wrow;
        const bool vec = ((a.o_t_ld | (int64_t)Sq | (int64_t)(uintptr_t)a.o_t) & 7) == 0;
#pragma unroll
        for (int pass = 0; pass < DT / 2; ++pass) {
#pragma unroll
          for (int X = 0; X < 2; ++X)
#pragma unroll
            for (int dd = 0; dd < 2; ++dd)
#pragma unroll
              for (int i = 0; i < 16; ++i) {
                const int d = 32 * dd + 8 * (i >> 2) + 4 * h + (i & 3);
                tt[d * C::TP + 32 * X + r] = f2bf(o[X][2 * pass + dd][i] * inv[X]);
              }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int seg = lane + 64 * k;  // 512 segments: d = seg / 8, tokens 8 (seg % 8) ..
            const int d = seg >> 3, t8 = seg & 7;
            const int tok0 = wrow + 8 * t8;
            bf16_t* dst = otb + (int64_t)(64 * pass + d) * a.o_t_ld + 8 * t8;
            const u16x8 v8 = *reinterpret_cast<const u16x8*>(tt + d * C::TP + 8 * t8);
            if (vec && tok0 + 8 <= Sq) {
              *reinterpret_cast<u16x8*>(dst) = v8;
            } else {
              for (int j = 0; j < 8 && tok0 + j < Sq; ++j) dst[j] = v8[j];
            }
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
      }
    }
  }
  // drain: no wave may end while its LDS-DMA is in flight into a ring another item could still read (none: every
  // issued tile was consumed), but keep the stores of the last epilogue ordered before exit
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if PICO_FWDP_STAMP
  FP_ST(9);
  ph[12] = __builtin_amdgcn_s_memtime() - tstart;
  ph[14] = __builtin_amdgcn_s_memrealtime();
  if (a.workspace && lane < 16) {
    unsigned long long v = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) v = lane == i ? ph[i] : v;
    ((unsigned long long*)a.workspace)[((int64_t)blockIdx.x * 4 + wave) * 16 + lane] = v;
  }
#endif
}
#undef FP_ST

template <int D>
int launch_fwdp(const pico_attn_args* a, hipStream_t s) {
  const int nJ = (int)((a->seqlen_q + PB - 1) / PB);
  const int64_t nbh = a->batch * a->heads_q;
  const float sl2 = a->softmax_scale * LOG2E;
  PICO_REQUIRE(sl2 > 0.f, "pico_attn_fwd: softmax_scale must be positive");
  // causal: pair blocks J and nJ-1-J in one persistent workgroup when that still fills every CU
  const int pairs = a->causal && nJ > 1 && nbh * ((nJ + 1) / 2) >= pico_num_cus() ? 1 : 0;
  const int64_t grid = nbh * (pairs ? (nJ + 1) / 2 : nJ);
  PICO_REQUIRE(grid < (1ll << 31), "pico_attn_fwd: grid too large");
  if (a->causal) {
    PICO_TRY(pico_launch(PICO_K_ATTN_FWD, "attn_fwd", attn_fwdp_kernel<D, true>, dim3((int)grid), dim3(256), 0, s, *a,
                         sl2, nJ, pairs));
  } else {
    PICO_TRY(pico_launch(PICO_K_ATTN_FWD, "attn_fwd", attn_fwdp_kernel<D, false>, dim3((int)grid), dim3(256), 0, s, *a,
                         sl2, nJ, pairs));
  }
  return 0;
}

}  // namespace

// The persistent kernel, opt-in (pico_select(PICO_SEL_ATTN_FWD, 1)), for the shapes it covers (head_dim 64, both
// lengths multiples of 64, equal lengths when causal); returns -1 when it does not apply. Not the default: measured
// SLOWER than the 32-row kernel at every shape (C2 causal 36.0 vs 27.9 us, non-causal 54.6 vs 45.8, S 4096 95.5 vs
// 80.3; profiles/r06_fwdp_check.jsonl). The phase stamps (PICO_FWDP_STAMP, profiles/r06_fwdp_stamps.jsonl) say why:
// at D = 64 the tile is VALU-issue bound and ONE wave per SIMD issues VALU at ~1 op / 4-5 cycles (two waves reach
// ~1 / 3.5): the four phases take 616 / 545 / 520 / 801 cycles for 8 MFMAs (256 cycles) each, 2,480 cycles per
// 64-row tile against the 32-row kernel's 2,720 per 64 rows at four waves per SIMD — no gain before the per-tile
// barrier (432, causal lockstep at the diagonal) and DMA issue (275), and 8 k cycles per item of Q prologue and
// epilogue that no co-resident workgroup overlaps. The structure pays where the MFMAs, not the softmax, bound the
// tile (the guide's D = 128); at D = 128 this kernel still spills (to do).
int pico_attn_fwdp(const pico_attn_args* a, hipStream_t s) {
  const int sel = pico_sel(PICO_SEL_ATTN_FWD);
  if (sel != 1) return -1;
  if (a->head_dim != 64) return -1;  // D = 128: spills at 512 registers (to do), the 32-row kernel
  if (a->seqlen_q % PN || a->seqlen_k % PN) return -1;
  if (a->causal && a->seqlen_q != a->seqlen_k) return -1;
  if (a->head_dim == 64) return launch_fwdp<64>(a, s);
  return launch_fwdp<128>(a, s);
}
