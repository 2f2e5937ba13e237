// Flash-attention forward for gfx950: causal / non-causal, GQA, bf16 MFMA, fp32 online softmax,
// fp32 LSE output.
//
// Replaces flash_attn_func(q, k, v, causal=True) (ref picotron/model.py:32-36,153; eager oracle
// F.scaled_dot_product_attention :156) and the ring block forward ring_attention_forward
// (ref picotron/context_parallel/context_parallel.py:112-128), which additionally returns the LSE.
//
// Structure (one workgroup = 4 waves = 128 query rows of one (batch, q-head); 64-key tiles):
//   * Q stays in registers for the whole sweep (B operand, 8 bf16 per lane per 16-wide k-step).
//   * K and V tiles are register-staged into a double-buffered, XOR-swizzled LDS image: the next
//     tile's global loads are issued before this tile's MFMAs and written to LDS after them (T14).
//   * Swapped product S^T = K * Q^T (v_mfma_f32_32x32x16_bf16): the accumulator has the query on
//     the lane and 16 keys in registers, so the online softmax is lane-local (one xor-32 shuffle
//     for the row max) and P^T is already the B operand of O^T += V^T * P^T (no LDS round trip);
//     V^T fragments come from ds_read_b64_tr_b16 on the row-major V image.
//   * Causal: tiles beyond the diagonal are never loaded; waves skip tiles entirely above their rows;
//     workgroups are issued heaviest-first over all heads (LPT order).
// FLOPs per (b, h): 4 * Sq * Sk * D (halved by the causal mask).
#include "attn_common.h"

namespace {

constexpr int BM = 128;  // query rows per workgroup (32 per wave)
constexpr int BN = 64;   // keys per tile

template <int D>
struct FwdSmem {
  char k[2][BN * D * 2];
  char v[2][BN * D * 2];
};

template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(const pico_attn_args a, float scale_log2) {
  constexpr int CPR = D / 8;                   // 16-byte chunks per row
  constexpr int CHUNKS_PER_THREAD = BN * CPR / 256;
  constexpr int KS = D / 16;                   // k-steps of the S^T product
  constexpr int DT = D / 32;                   // 32-wide output tiles of O^T
  __shared__ __attribute__((aligned(16))) FwdSmem<D> sm;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (scalar branches)
  const int r = lane & 31, h = lane >> 5;

  // LPT order: heaviest query blocks of every head first.
  const int nmb = (int)((a.seqlen_q + BM - 1) / BM);
  const int nbh = (int)(a.batch * a.heads_q);
  const int lin = blockIdx.x;
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
    const bool ok = my_q < Sq;
    const bf16_t* qp = qg + (int64_t)min(my_q, Sq - 1) * a.q_strides[1] + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(qp + 16 * ks);
      qf[ks] = __builtin_bit_cast(bf16x8, ok ? v : (u16x8)0);
    }
  }

  // number of key tiles this workgroup visits
  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + BM);
  const int ntiles = (kend + BN - 1) / BN;

  // ---- register staging of K/V tiles ----
  // Loads are issued unconditionally from a clamped row; the zero-fill of rows past Sk is applied
  // when the registers are written to LDS, so no wait is forced right after the loads.
  u16x8 kreg[CHUNKS_PER_THREAD], vreg[CHUNKS_PER_THREAD];
  auto gload = [&](int tile) {
#pragma unroll
    for (int c = 0; c < CHUNKS_PER_THREAD; ++c) {
      const int id = threadIdx.x + 256 * c;
      const int row = id / CPR, ch = id % CPR;
      const int kc = min(tile * BN + row, Sk - 1);
      kreg[c] = *reinterpret_cast<const u16x8*>(kg + (int64_t)kc * ksd + ch * 8);
      vreg[c] = *reinterpret_cast<const u16x8*>(vg + (int64_t)kc * vsd + ch * 8);
    }
  };
  auto swrite = [&](int buf, int tile) {
#pragma unroll
    for (int c = 0; c < CHUNKS_PER_THREAD; ++c) {
      const int id = threadIdx.x + 256 * c;
      const int row = id / CPR, ch = id % CPR;
      const bool ok = tile * BN + row < Sk;
      const int off = lds_off<D>(row, ch);
      *reinterpret_cast<u16x8*>(sm.k[buf] + off) = ok ? kreg[c] : (u16x8)0;
      *reinterpret_cast<u16x8*>(sm.v[buf] + off) = ok ? vreg[c] : (u16x8)0;
    }
  };

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = (f32x16)0.f;
  float m_i = -INFINITY, l_i = 0.f;

  if (ntiles > 0) {
    gload(0);
    swrite(0, 0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const bool more = t + 1 < ntiles;
    if (more) gload(t + 1);
    const int n0 = t * BN;
    // whole tile above this wave's rows (causal) -> nothing to do for this wave
    const bool active = !CAUSAL || n0 <= qw + 31;
    if (active) {
      const char* kb = sm.k[buf];
      const char* vb = sm.v[buf];
      f32x16 s[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] = (f32x16)0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 kf = lds_read_b128(kb, lds_off<D>(kt * 32 + r, 2 * ks + h));
          s[kt] = mfma32(kf, qf[ks], s[kt]);
        }
      }
      // scale + mask; lane holds query my_q and keys n0 + 32 kt + acc_row(i, h)
      const bool need_mask = (n0 + BN > Sk) || (CAUSAL && n0 + BN - 1 > qw);
      float mloc = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float x = s[kt][i] * scale_log2;
          if (need_mask) {
            const int key = n0 + kt * 32 + acc_row(i, h);
            x = (key >= Sk || (CAUSAL && key > my_q)) ? -INFINITY : x;
          }
          s[kt][i] = x;
          mloc = fmaxf(mloc, x);
        }
      }
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float m_new = fmaxf(m_i, mloc);
      const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
      const float alpha = fast_exp2(m_i - m_use);
      float lsum = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = fast_exp2(s[kt][i] - m_use);
          s[kt][i] = p;
          lsum += p;
        }
      }
      l_i = l_i * alpha + lsum;
      m_i = m_new;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      // O^T[dt] += V^T * P^T : A = V^T via transposed LDS read, B = packed P^T registers
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          float pv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) pv[j] = s[kt][8 * st + j];
          const bf16x8 pf = pack_frag(pv);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const bf16x8 vf = lds_read_tr32<D>(vb, kt * 32 + 16 * st, dt * 32, lane);
            o[dt] = mfma32(vf, pf, o[dt]);
          }
        }
      }
    }
    if (more) swrite(buf ^ 1, t + 1);
    __syncthreads();
  }

  // ---- epilogue: O = O^T / l, LSE = (m + log2 l) * ln2 ----
  const float l_tot = l_i + __shfl_xor(l_i, 32, 64);
  if (my_q < Sq) {
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    bf16_t* op = (bf16_t*)a.o + b * a.o_strides[0] + hq * a.o_strides[2] + (int64_t)my_q * a.o_strides[1];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // registers 4g..4g+3 hold d = 32 dt + 8 g + 4 h + 0..3
        u16x4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = f2bf(o[dt][4 * g + j] * inv);
        *reinterpret_cast<u16x4*>(op + 32 * dt + 8 * g + 4 * h) = w;
      }
    }
    if (h == 0) {
      const float lse = l_tot > 0.f ? (m_i + __log2f(l_tot)) * LN2 : -INFINITY;
      a.lse[((int64_t)b * a.heads_q + hq) * Sq + my_q] = lse;
    }
  }
}

template <int D>
int launch_fwd(const pico_attn_args* a, hipStream_t s) {
  const int nmb = (int)((a->seqlen_q + BM - 1) / BM);
  const int64_t nblk = (int64_t)nmb * a->batch * a->heads_q;
  PICO_REQUIRE(nblk < (1ll << 31), "pico_attn_fwd: grid too large");
  const float sl2 = a->softmax_scale * LOG2E;
  if (a->causal) {
    PICO_LAUNCH(PICO_K_ATTN_FWD, "attn_fwd", s, attn_fwd_kernel<D, true><<<(int)nblk, 256, 0, s>>>(*a, sl2));
  } else {
    PICO_LAUNCH(PICO_K_ATTN_FWD, "attn_fwd", s, attn_fwd_kernel<D, false><<<(int)nblk, 256, 0, s>>>(*a, sl2));
  }
  return 0;
}

}  // namespace

int pico_attn_check_common(const pico_attn_args* a, const char* op);

extern "C" int pico_attn_fwd(const pico_attn_args* a, void* stream) {
  int rc = pico_attn_check_common(a, "pico_attn_fwd");
  if (rc) return rc;
  PICO_REQUIRE(a->o && a->lse, "pico_attn_fwd: null output");
  if (a->batch == 0 || a->seqlen_q == 0 || a->heads_q == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (a->head_dim == 64) return launch_fwd<64>(a, s);
  return launch_fwd<128>(a, s);
}
