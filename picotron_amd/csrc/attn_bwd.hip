// Flash-attention backward for gfx950: dQ, dK, dV from (Q, K, V, O, dO, LSE); causal / non-causal,
// GQA, bf16 MFMA with fp32 accumulation.
//
// Replaces flash-attn's backward of flash_attn_func (ref picotron/model.py:36) and the ring block
// backward ring_attention_backward (ref picotron/context_parallel/context_parallel.py:130-155),
// which recomputes P from the (global) O and LSE:  P = exp(scale*QK^T - LSE), dV = P^T dO,
// dP = dO V^T, delta = rowsum(dO * O), dS = P * (dP - delta), dQ = scale * dS K, dK = scale * dS^T Q.
//
// Structure: one workgroup = 8 waves = 256 keys of one (batch, kv-head); wave w owns keys
// 32w..32w+31 with the key on the MFMA lane, keeps dK^T/dV^T of its keys in accumulators for the
// whole sweep over (q-heads of the group) x (32-row query tiles), so dK/dV need no cross-workgroup
// sum. S and dP are computed with the key on the lane, which makes their accumulators directly the
// A operand of dV = P^T dO and dK = dS^T Q (the dO / Q tile is read transposed with
// ds_read_b64_tr_b16). dS crosses LDS once for dQ = dS K, computed as 16x16 tiles over all 256 keys
// over all 256 keys, and each workgroup writes its fp32 dQ partial with plain stores into its key
// block's slab; attn_bwd_dq_kernel sums the slabs in key-block order (no atomics: plain stores run
// ~4-5x the chip's float-atomic rate, and the result is bitwise reproducible).
// FLOPs per (b, h): 10 * Sq * Sk * D (halved by the causal mask); 2.5x the forward.
#include "attn_common.h"

namespace {

constexpr int BK = 256;  // keys per workgroup
constexpr int BQ = 32;   // query rows per tile

template <int D>
struct BwdSmem {
  char k[BK * D * 2];        // K image [key][d] (B operand of S, transposed B operand of dQ)
  char q[2][BQ * D * 2];     // Q tiles [q][d], double-buffered
  char dout[2][BQ * D * 2];  // dO tiles [q][d], double-buffered
  char ds[BQ * BK * 2];      // dS image [q][key], chunk-swizzled
  float lse2[2][BQ];         // LSE * log2(e)
  float delta[2][BQ];
};

PICO_DEV int ds_off(int q, int key) {
  // 512-B rows of 32 chunks; low 4 chunk bits XOR (q & 15)
  const int chunk = key >> 3;
  return q * 512 + 16 * (chunk ^ (q & 15)) + (key & 7) * 2;
}

// delta[b, h, q] = sum_d dO * O  (fp32)
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const pico_attn_args a, float* __restrict__ delta) {
  constexpr int LPR = D / 8;  // lanes per row (8 bf16 each)
  const int64_t rows = a.batch * a.seqlen_q * a.heads_q;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  if (row >= rows) return;
  const int hq = (int)(row % a.heads_q);
  const int64_t bq = row / a.heads_q;
  const int q = (int)(bq % a.seqlen_q);
  const int b = (int)(bq / a.seqlen_q);
  const u16x8 ov = *reinterpret_cast<const u16x8*>((const bf16_t*)a.o + b * a.o_strides[0] + q * a.o_strides[1] +
                                                   hq * a.o_strides[2] + sub * 8);
  const u16x8 dv = *reinterpret_cast<const u16x8*>((const bf16_t*)a.dout + b * a.do_strides[0] +
                                                   q * a.do_strides[1] + hq * a.do_strides[2] + sub * 8);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += bf2f(ov[j]) * bf2f(dv[j]);
#pragma unroll
  for (int o = LPR / 2; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if (sub == 0) delta[((int64_t)b * a.heads_q + hq) * a.seqlen_q + q] = s;
}

// Main backward kernel. Per tile (32 query rows of one q-head):
//   load-ahead: the NEXT tile's Q/dO/LSE/delta go global -> registers before this tile's MFMAs and
//   registers -> the other LDS buffer after them (T14), so HBM latency hides under compute;
//   S, dP (MFMA) -> P, dS (VALU) -> dV += P^T dO, dK += dS^T Q (MFMA) -> dS to LDS -> barrier ->
//   dQ partial = dS K over the workgroup's 256 keys (16x16 tiles, one per wave) -> plain fp32 stores
//   into this key block's slab (summed by attn_bwd_dq_kernel in a fixed order: no atomics,
//   bitwise reproducible) -> barrier.
template <int D, bool CAUSAL>
__global__ __launch_bounds__(512, 2) void attn_bwd_kernel(const pico_attn_args a, float scale, float scale_log2,
                                                          const float* __restrict__ delta_g, float* __restrict__ dq_part,
                                                          int64_t slab) {
  constexpr int CPR = D / 8;
  constexpr int KS = D / 16;
  constexpr int DT = D / 32;
  constexpr int NCH = 2 * BQ * CPR / 512;  // staged 16-B chunks per thread (Q and dO)
  __shared__ __attribute__((aligned(16))) BwdSmem<D> sm;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (scalar branches)
  const int r = lane & 31, h = lane >> 5;
  const int Sq = (int)a.seqlen_q, Sk = (int)a.seqlen_k;
  const int Hq = (int)a.heads_q;
  const int G = (int)(a.heads_q / a.heads_kv);

  // heaviest key blocks first (causal: block 0 sees every query)
  const int nbh = (int)(a.batch * a.heads_kv);
  const int kb = blockIdx.x / nbh;
  const int bh = blockIdx.x % nbh;
  const int b = bh / (int)a.heads_kv;
  const int hk = bh % (int)a.heads_kv;

  const int k0 = kb * BK;
  const int kw = k0 + 32 * wave;  // this wave's first key
  const int my_key = kw + r;

  const bf16_t* kg = (const bf16_t*)a.k + b * a.k_strides[0] + hk * a.k_strides[2];
  const bf16_t* vg = (const bf16_t*)a.v + b * a.v_strides[0] + hk * a.v_strides[2];

  // ---- K block -> LDS image; V fragments -> registers (B operand of dP = dO V^T) ----
  for (int id = threadIdx.x; id < BK * CPR; id += 512) {
    const int row = id / CPR, ch = id % CPR;
    const int key = k0 + row;
    const u16x8 v = *reinterpret_cast<const u16x8*>(kg + (int64_t)min(key, Sk - 1) * a.k_strides[1] + ch * 8);
    *reinterpret_cast<u16x8*>(sm.k + lds_off<D>(row, ch)) = key < Sk ? v : (u16x8)0;
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

  const int qstart = CAUSAL ? k0 : 0;  // k0 is a multiple of BQ
  const int nqt = Sq > qstart ? (Sq - qstart + BQ - 1) / BQ : 0;
  const int ntiles = G * nqt;

  // ---- tile staging (global -> registers -> LDS) ----
  // Thread roles are fixed for the whole sweep: chunk j of this thread stages Q (which == 0) or dO
  // rows; the role is wave-uniform (D = 64: waves 0-3 vs 4-7; D = 128: by j), so base pointers and
  // strides are selected once, in scalar registers. Loads read a clamped row unconditionally; the
  // zero-fill of padded rows is applied at the LDS write so nothing waits right after a load.
  const bf16_t* stg_base[NCH];
  int64_t stg_hs[NCH], stg_ss[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int which = __builtin_amdgcn_readfirstlane((int)((threadIdx.x + 512 * j) / (BQ * CPR)));
    stg_base[j] = which == 0 ? (const bf16_t*)a.q + b * a.q_strides[0] : (const bf16_t*)a.dout + b * a.do_strides[0];
    stg_hs[j] = which == 0 ? a.q_strides[2] : a.do_strides[2];
    stg_ss[j] = which == 0 ? a.q_strides[1] : a.do_strides[1];
  }
  const float* stg_cbase = threadIdx.x < BQ ? a.lse : delta_g;
  u16x8 stg[NCH];
  float stg_c = 0.f;
  auto gload = [&](int t) {
    const int hq = hk * G + t / nqt;
    const int q0 = qstart + (t % nqt) * BQ;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int rem = (threadIdx.x + 512 * j) % (BQ * CPR);
      const int row = rem / CPR, ch = rem % CPR;
      const int qc = min(q0 + row, Sq - 1);
      stg[j] = *reinterpret_cast<const u16x8*>(stg_base[j] + hq * stg_hs[j] + (int64_t)qc * stg_ss[j] + ch * 8);
    }
    const int qc = min(q0 + (int)(threadIdx.x & (BQ - 1)), Sq - 1);
    stg_c = stg_cbase[((int64_t)b * Hq + hq) * Sq + qc];
  };
  auto swrite = [&](int buf, int t) {
    const int q0 = qstart + (t % nqt) * BQ;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c = threadIdx.x + 512 * j;
      const int which = c / (BQ * CPR), rem = c % (BQ * CPR);
      const int row = rem / CPR, ch = rem % CPR;
      char* dst = which == 0 ? sm.q[buf] : sm.dout[buf];
      *reinterpret_cast<u16x8*>(dst + lds_off<D>(row, ch)) = q0 + row < Sq ? stg[j] : (u16x8)0;
    }
    const bool ok = q0 + (int)(threadIdx.x & (BQ - 1)) < Sq;
    if (threadIdx.x < BQ)
      sm.lse2[buf][threadIdx.x] = ok ? stg_c * LOG2E : INFINITY;  // +inf LSE -> P = 0 for padded rows
    else if (threadIdx.x < 2 * BQ)
      sm.delta[buf][threadIdx.x - BQ] = ok ? stg_c : 0.f;
  };

  if (ntiles > 0) {
    gload(0);
    swrite(0, 0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    const int hq = hk * G + t / nqt;
    const int q0 = qstart + (t % nqt) * BQ;
    const bool more = t + 1 < ntiles;
    if (more) gload(t + 1);

    const bool active = !CAUSAL || kw <= q0 + BQ - 1;
    if (active) {
      const char* qs = sm.q[buf];
      const char* dos = sm.dout[buf];
      // S[q][key] and dP[q][key]: A = Q / dO rows (LDS), B = K^T (LDS) / V^T (registers)
      f32x16 s = (f32x16)0.f, dp = (f32x16)0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 qa = lds_read_b128(qs, lds_off<D>(r, 2 * ks + h));
        const bf16x8 kbf = lds_read_b128(sm.k, lds_off<D>(32 * wave + r, 2 * ks + h));
        s = mfma32(qa, kbf, s);
        const bf16x8 da = lds_read_b128(dos, lds_off<D>(r, 2 * ks + h));
        dp = mfma32(da, vf[ks], dp);
      }
      // P = exp2(S * scale*log2e - LSE*log2e) (in s), dS = P * (dP - delta) (in dp); lane: key my_key
      const bool need_mask = (CAUSAL && kw + 31 > q0) || (k0 + BK > Sk);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qi = acc_row(i, h);
        float pv = fast_exp2(s[i] * scale_log2 - sm.lse2[buf][qi]);
        if (need_mask) pv = ((CAUSAL && my_key > q0 + qi) || my_key >= Sk) ? 0.f : pv;
        s[i] = pv;
        dp[i] = pv * (dp[i] - sm.delta[buf][qi]);
      }
      // dV[key][d] += P^T dO ; dK[key][d] += dS^T Q   (k index = query rows of the tile)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        float pv[8], sv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pv[j] = s[8 * st + j];
          sv[j] = dp[8 * st + j];
        }
        const bf16x8 pf = pack_frag(pv);
        const bf16x8 sf = pack_frag(sv);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const bf16x8 dof = lds_read_tr32<D>(dos, 16 * st, 32 * dt, lane);
          dv[dt] = mfma32(pf, dof, dv[dt]);
          const bf16x8 qf = lds_read_tr32<D>(qs, 16 * st, 32 * dt, lane);
          dk[dt] = mfma32(sf, qf, dk[dt]);
        }
      }
      // dS (bf16) -> LDS image [q][key] for dQ
#pragma unroll
      for (int i = 0; i < 16; ++i)
        *reinterpret_cast<bf16_t*>(sm.ds + ds_off(acc_row(i, h), 32 * wave + r)) = f2bf(dp[i]);
    }
    __syncthreads();  // dS visible

    // ---- dQ partial [q][d] = scale * dS[q][:] K[:][d] over this block's keys: 16x16 tiles ----
    {
      constexpr int NT = (BQ / 16) * (D / 16);
      int kmax = min(BK, Sk - k0);
      if (CAUSAL) kmax = min(kmax, ((q0 + BQ - 1 - k0) / 32 + 1) * 32);
      kmax = (kmax + 31) & ~31;
#pragma unroll
      for (int tt = 0; tt < NT / 8; ++tt) {
        const int tl = wave + 8 * tt;
        const int qi = tl / (D / 16), di = tl % (D / 16);
        f32x4 acc = (f32x4)0.f;
        for (int kk = 0; kk < kmax; kk += 32) {
          const bf16x8 af = lds_read_b128(sm.ds, ds_off(qi * 16 + (lane & 15), kk + 8 * (lane >> 4)));
          const bf16x8 bf = lds_read_tr16<D>(sm.k, kk, di * 16, lane);
          acc = mfma16(af, bf, acc);
        }
        float* dst = dq_part + kb * slab + (int64_t)b * Sq * Hq * D + hq * D + di * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int q = q0 + qi * 16 + 4 * (lane >> 4) + j;
          if (q < Sq) dst[(int64_t)q * Hq * D] = acc[j] * scale;
        }
      }
    }
    if (more) swrite(buf ^ 1, t + 1);
    __syncthreads();  // next tile staged; dS reads done
  }

  // ---- epilogue: dK = scale * acc, dV = acc; lane holds d = 32 dt + r, keys kw + acc_row(i, h) ----
  bf16_t* dkg = (bf16_t*)a.dk + b * a.dk_strides[0] + hk * a.dk_strides[2];
  bf16_t* dvg = (bf16_t*)a.dv + b * a.dv_strides[0] + hk * a.dv_strides[2];
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
}

// dq[b, q, h, :] = sum over key blocks kb (causal: kb * 256 <= q) of the fp32 partial slabs, summed in
// kb order (deterministic). Writes bf16 (strided), or ADDS into an fp32 accumulator.
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(const pico_attn_args a, const float* __restrict__ dq_part,
                                                          int64_t slab, int nkb, int f32acc) {
  constexpr int LPR = D / 8;
  const int64_t rows = a.batch * a.seqlen_q * a.heads_q;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;
  const int sub = threadIdx.x % LPR;
  if (row >= rows) return;
  const int hq = (int)(row % a.heads_q);
  const int64_t bq = row / a.heads_q;
  const int q = (int)(bq % a.seqlen_q);
  const int b = (int)(bq / a.seqlen_q);
  const int last = CAUSAL ? min(nkb - 1, q / BK) : nkb - 1;
  f32x4 x0 = (f32x4)0.f, x1 = (f32x4)0.f;
  for (int k = 0; k <= last; ++k) {
    const f32x4* src = reinterpret_cast<const f32x4*>(dq_part + k * slab + row * D + sub * 8);
    x0 += src[0];
    x1 += src[1];
  }
  if (f32acc) {
    float* dst = (float*)a.dq + b * a.dq_strides[0] + q * a.dq_strides[1] + hq * a.dq_strides[2] + sub * 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dst[j] += x0[j];
      dst[4 + j] += x1[j];
    }
    return;
  }
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = f2bf(x0[j]);
    o[4 + j] = f2bf(x1[j]);
  }
  *reinterpret_cast<u16x8*>((bf16_t*)a.dq + b * a.dq_strides[0] + q * a.dq_strides[1] + hq * a.dq_strides[2] +
                            sub * 8) = o;
}

int64_t delta_floats(const pico_attn_args* a) {
  const int64_t nrow = a->batch * a->heads_q * a->seqlen_q;
  return ((nrow + 63) / 64) * 64;
}

template <int D>
int launch_bwd(const pico_attn_args* a, hipStream_t s) {
  const int f32acc = (a->flags & PICO_ATTN_DQ_F32_ACCUM) != 0;
  float* delta = (float*)a->workspace;
  float* dq_part = delta + delta_floats(a);
  const int64_t slab = a->batch * a->seqlen_q * a->heads_q * D;
  const int64_t rows = a->batch * a->seqlen_q * a->heads_q;
  const int row_blocks = pico_cdiv(rows * (D / 8), 256);
  PICO_LAUNCH(PICO_K_ATTN_BWD_PRE, "attn_bwd_pre", s, attn_bwd_pre_kernel<D><<<row_blocks, 256, 0, s>>>(*a, delta));
  const int nkb = (int)((a->seqlen_k + BK - 1) / BK);
  const int64_t nblk = (int64_t)nkb * a->batch * a->heads_kv;
  const float sl2 = a->softmax_scale * LOG2E;
  if (nblk > 0) {
    if (a->causal) {
      PICO_LAUNCH(PICO_K_ATTN_BWD, "attn_bwd", s,
                  attn_bwd_kernel<D, true><<<(int)nblk, 512, 0, s>>>(*a, a->softmax_scale, sl2, delta, dq_part, slab));
    } else {
      PICO_LAUNCH(PICO_K_ATTN_BWD, "attn_bwd", s,
                  attn_bwd_kernel<D, false><<<(int)nblk, 512, 0, s>>>(*a, a->softmax_scale, sl2, delta, dq_part, slab));
    }
  }
  if (a->causal) {
    PICO_LAUNCH(PICO_K_ATTN_BWD_DQ, "attn_bwd_dq", s,
                attn_bwd_dq_kernel<D, true><<<row_blocks, 256, 0, s>>>(*a, dq_part, slab, nkb, f32acc));
  } else {
    PICO_LAUNCH(PICO_K_ATTN_BWD_DQ, "attn_bwd_dq", s,
                attn_bwd_dq_kernel<D, false><<<row_blocks, 256, 0, s>>>(*a, dq_part, slab, nkb, f32acc));
  }
  return 0;
}

}  // namespace

// Shared argument validation for forward and backward.
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
  // delta [B*Hq*Sq] fp32 + one fp32 dQ partial slab [B, Sq, Hq, D] per 256-key block
  const int64_t nkb = (a->seqlen_k + BK - 1) / BK;
  return (delta_floats(a) + nkb * a->batch * a->seqlen_q * a->heads_q * a->head_dim) * 4;
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
  if (a->batch == 0 || a->seqlen_q == 0 || a->heads_q == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (a->head_dim == 64) return launch_bwd<64>(a, s);
  return launch_bwd<128>(a, s);
}

}  // extern "C"
