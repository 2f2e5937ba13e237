// Shared pieces of the gfx950 flash-attention forward/backward kernels.
#pragma once
#include "common.h"

typedef __attribute__((address_space(3))) i16x4 lds_i16x4;

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// MFMA 32x32x16 bf16 -> fp32 (per wave: D[32x32] += A[32x16] * B[16x32]).
// Operand maps (cdna_hip_programming.md §3): lane l (r = l&31, h = l>>5) holds A[r][8h+j] and
// B[8h+j][r], j = 0..7; the accumulator holds D[(reg&3) + 8*(reg>>2) + 4*h][r].
PICO_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// MFMA 16x16x32 bf16: lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15]; D[4(l>>4)+reg][l&15].
PICO_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Accumulator row index of register `reg` for lane-half h (32x32 layout).
PICO_DEV int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// ---- LDS tile images -------------------------------------------------------------------
// A tile of R rows x D bf16 is stored row-major with its 16-byte chunks XOR-swizzled per row so
// that both access kinds used on it are bank-conflict free (MI355X_MICROARCH.md §LDS):
//   * ds_read_b128 of one chunk from 16 different rows (MFMA operand with the row on the lane);
//   * ds_read_b64_tr_b16 of 4 consecutive rows x 4 consecutive chunks (transposed operand).
// D = 128 (256-B rows): chunk ^ (((r & 3) << 2) | ((r >> 2) & 3))   (cdna_hip_programming.md T10 (b))
// D = 64  (128-B rows, two rows per bank row): chunk ^ g((r >> 1) & 7), g(y) = y ^ ((y & 1) << 2)
template <int D>
PICO_DEV int lds_off(int row, int chunk) {
  if constexpr (D == 128) {
    return row * 256 + 16 * (chunk ^ (((row & 3) << 2) | ((row >> 2) & 3)));
  } else {
    static_assert(D == 64, "head_dim 64 or 128");
    const int y = (row >> 1) & 7;
    return row * 128 + 16 * (chunk ^ (y ^ ((y & 1) << 2)));
  }
}

PICO_DEV bf16x8 lds_read_b128(const char* base, int off) {
  return *reinterpret_cast<const bf16x8*>(base + off);
}

// Transposed operand read: for 32x32x16 with the k index running over tile ROWS.
// Returns, for lane (r = lane&31 -> column col0 + r, h = lane>>5), the 8 bf16 elements
// T[row0 + 8*(j>>2) + 4*h + (j&3)][col0 + r], j = 0..7, via two ds_read_b64_tr_b16.
// (This is exactly the k-permutation of an accumulator used as the other operand, §3.)
template <int D>
PICO_DEV bf16x8 lds_read_tr32(const char* base, int row0, int col0, int lane) {
  const int g = lane >> 4;  // 16-lane group
  const int i = lane & 15;
  const int h = g >> 1;
  const int q = i >> 2, p = i & 3;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  const int chunk = col >> 3, sub = (col & 7) * 2;
  const int r0 = row0 + 4 * h + q;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + lds_off<D>(r0, chunk) + sub));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + lds_off<D>(r0 + 8, chunk) + sub));
  typedef __attribute__((ext_vector_type(8))) short i16x8;
  i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Transposed operand read for 16x16x32 with k over tile ROWS: lane l gets
// T[row0 + 8*(l>>4) + j][col0 + (l&15)], j = 0..7 (natural k order).
template <int D>
PICO_DEV bf16x8 lds_read_tr16(const char* base, int row0, int col0, int lane) {
  const int g = lane >> 4;
  const int i = lane & 15;
  const int q = i >> 2, p = i & 3;
  const int col = col0 + 4 * p;
  const int chunk = col >> 3, sub = (col & 7) * 2;
  const int r0 = row0 + 8 * g + q;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + lds_off<D>(r0, chunk) + sub));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + lds_off<D>(r0 + 4, chunk) + sub));
  typedef __attribute__((ext_vector_type(8))) short i16x8;
  i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Transposed 32x32x16 operand from a per-lane address (the caller's layout supplies, for lane
// (g = lane>>4, q = (lane&15)>>2, p = lane&3), the byte address of row 4*(lane>>5) + q, columns
// 16*(g&1) + 4p .. +3 of the block): two ds_read_b64_tr_b16, the second `hi` bytes further (8 rows).
// Result element j of lane (r, h) = T[8*(j>>2) + 4h + (j&3)][r]  (see lds_read_tr32).
PICO_DEV bf16x8 lds_read_tr_rows(const char* p, int hi) {
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)p);
  const i16x4 up = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(p + hi));
  typedef __attribute__((ext_vector_type(8))) short i16x8;
  i16x8 v = {lo[0], lo[1], lo[2], lo[3], up[0], up[1], up[2], up[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// ds_read_b64_tr_b16 at an LDS byte address + immediate (inline asm: hipcc re-bases DS address
// chains onto negative offsets it cannot fold, costing a VALU add per read). The compiler does not
// track these reads: consume them only after lds_wait_all().
template <int OFF>
PICO_DEV i16x4 ds_tr16_imm(unsigned addr) {
  static_assert(OFF >= 0 && OFF < 65536, "DS offset is 16-bit unsigned");
  i16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
  return r;
}
// Two of them = one 32x32x16 operand (rows +0..3 at OFF, +8..11 at OFF + HI), see lds_read_tr_rows.
template <int OFF, int HI>
PICO_DEV bf16x8 tr_operand_imm(unsigned addr) {
  const i16x4 lo = ds_tr16_imm<OFF>(addr);
  const i16x4 up = ds_tr16_imm<OFF + HI>(addr);
  typedef __attribute__((ext_vector_type(8))) short i16x8;
  i16x8 v = {lo[0], lo[1], lo[2], lo[3], up[0], up[1], up[2], up[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// Wait for every outstanding LDS read (incl. the inline-asm ones) and stop the scheduler from
// hoisting their consumers above the wait (cdna_hip_programming.md §5.4 rule 18).
PICO_DEV void lds_wait_all() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
PICO_DEV unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}

// 8 fp32 accumulator registers -> bf16x8 MFMA operand fragment (round to nearest even).
PICO_DEV bf16x8 pack_frag(const float* v) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
  return r;
}

// The same from 8 floats with one v_cvt_pk_bf16_f32 per pair (element order kept; no lane shuffles).
PICO_DEV bf16x8 pack_bf16x8(const float* v) {
  typedef __attribute__((ext_vector_type(2))) float f32x2;
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  const bf16x2 p0 = __builtin_convertvector((f32x2){v[0], v[1]}, bf16x2);
  const bf16x2 p1 = __builtin_convertvector((f32x2){v[2], v[3]}, bf16x2);
  const bf16x2 p2 = __builtin_convertvector((f32x2){v[4], v[5]}, bf16x2);
  const bf16x2 p3 = __builtin_convertvector((f32x2){v[6], v[7]}, bf16x2);
  const bf16x4 lo = __builtin_shufflevector(p0, p1, 0, 1, 2, 3);
  const bf16x4 hi = __builtin_shufflevector(p2, p3, 0, 1, 2, 3);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

PICO_DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// ---- shared by the backward kernels (attn_bwd.hip, attn_bwd_split.hip) ----

// One LDS-DMA piece (16 B per lane, lane-linear at the wave-uniform LDS byte address lds_base) issued
// from inline asm: the compiler does not see it as an LDS write, so it inserts none of its
// conservative `s_waitcnt vmcnt(0)` before the loop's LDS reads and writes (which would expose the
// full HBM latency of the piece just issued, every tile). The kernel's counted waits + barrier order
// the pieces against their readers; ring slots are never touched while a piece for them is in flight.
// Address = wave-uniform base (SGPR pair) + per-lane 32-bit byte offset.
PICO_DEV void dma_piece(const void* base, unsigned voff, unsigned lds_base) {
  const uint64_t p = (uint64_t)(uintptr_t)base;  // wave-uniform by construction; make it an SGPR pair
  const uint64_t sbase = (uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)p) |
                         ((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(p >> 32)) << 32);
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_base) : "memory");
}

// Workgroup barrier without the fence __syncthreads() implies (whose release semantics make the
// compiler drain vmcnt(0) — the in-flight DMA and dQ stores — before every barrier). LDS writes are
// drained (lgkmcnt(0)); the asm memory clobbers keep memory accesses from moving across it.
PICO_DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the immediate must be a constant)
PICO_DEV void wait_vmcnt(int n) {
  switch (n) {
#define PICO_VMCNT_CASE(N) \
  case N:                  \
    asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); \
    break;
    PICO_VMCNT_CASE(1) PICO_VMCNT_CASE(2) PICO_VMCNT_CASE(3) PICO_VMCNT_CASE(4) PICO_VMCNT_CASE(5)
    PICO_VMCNT_CASE(6) PICO_VMCNT_CASE(7) PICO_VMCNT_CASE(8) PICO_VMCNT_CASE(9) PICO_VMCNT_CASE(10)
    PICO_VMCNT_CASE(11) PICO_VMCNT_CASE(12) PICO_VMCNT_CASE(13) PICO_VMCNT_CASE(14) PICO_VMCNT_CASE(15)
    PICO_VMCNT_CASE(16) PICO_VMCNT_CASE(17) PICO_VMCNT_CASE(18) PICO_VMCNT_CASE(19) PICO_VMCNT_CASE(20)
#undef PICO_VMCNT_CASE
    default:
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// Stores one lane's 32x32 accumulator column(s) as a bf16 row with 16-byte stores: lane (r, h) holds
// d = 32 dt + 8 g + 4 h + j (j < 4) of row r, so lanes l and l + 32 (the same row) exchange half-chunks
// with v_permlane32_swap until each holds 8 consecutive d: lane h = 0 the even g, lane h = 1 the odd g
// (half the store instructions of the 8-byte form; cdna_hip_programming.md T21). Every lane of the wave
// must execute it (permlane: EXEC all ones); `ok` predicates only the stores.
template <int DT, typename Get>
PICO_DEV void store_row_bf16_x16(bf16_t* row, int h, bool ok, Get get) {
  typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      u16x4 e, o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        e[j] = f2bf(get(dt, 4 * (2 * p) + j));
        o[j] = f2bf(get(dt, 4 * (2 * p + 1) + j));
      }
      u32x2 ev = __builtin_bit_cast(u32x2, e), ov = __builtin_bit_cast(u32x2, o);
#pragma unroll
      for (int w = 0; w < 2; ++w) {
        const auto rr = __builtin_amdgcn_permlane32_swap(ev[w], ov[w], false, false);
        ev[w] = rr[0];
        ov[w] = rr[1];
      }
      const u32x4 out = {ev[0], ev[1], ov[0], ov[1]};
      if (ok) *reinterpret_cast<u32x4*>(row + 32 * dt + 8 * (2 * p + h)) = out;
    }
}

// XOR applied to the 16-B chunk index of image row `row` (see lds_off in attn_common.h)
template <int D>
PICO_DEV int swz(int row) {
  if constexpr (D == 128) return ((row & 3) << 2) | ((row >> 2) & 3);
  const int y = (row >> 1) & 7;
  return y ^ ((y & 1) << 2);
}

// rotate-half RoPE backward (rotation by -theta) of the pair (x[d], x[d + D/2]), d = i0 + j, j < 8, at
// sequence position pos: x1' = x1 c + x2 s, x2' = x2 c - x1 s (pico_rope with conjugate = 1)
PICO_DEV void rope_bwd8(const pico_attn_args& a, int pos, int i0, float* x1, float* x2) {
  const u16x8 c = *reinterpret_cast<const u16x8*>((const bf16_t*)a.rope_cos + (int64_t)pos * a.rope_stride + i0);
  const u16x8 sn = *reinterpret_cast<const u16x8*>((const bf16_t*)a.rope_sin + (int64_t)pos * a.rope_stride + i0);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float cf = bf2f(c[j]), sf = bf2f(sn[j]), u = x1[j], w = x2[j];
    x1[j] = u * cf + w * sf;
    x2[j] = w * cf - u * sf;
  }
}

// dK / dV [b, key, hk, :] = sum over the hsplit workgroups' fp32 partials (fixed order) -> bf16 (strided);
// dK optionally rotated back (PICO_ATTN_ROPE_BWD). Thread layout as attn_bwd_dq_kernel.
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(const pico_attn_args a, const float* __restrict__ dkv_part,
                                                           int hsplit) {
  constexpr int TPR = D / 16;
  const int64_t part = a.batch * a.seqlen_k * a.heads_kv * D;
  const int64_t rows = a.batch * a.seqlen_k * a.heads_kv;
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / TPR;
  const int d0 = (threadIdx.x % TPR) * 8;
  if (row >= rows) return;
  const int hk = (int)(row % a.heads_kv);
  const int64_t bk = row / a.heads_kv;
  const int key = (int)(bk % a.seqlen_k);
  const int b = (int)(bk / a.seqlen_k);
  for (int which = 0; which < 2; ++which) {
    float x1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, x2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int hs = 0; hs < hsplit; ++hs) {
      const float* src = dkv_part + (2 * hs + which) * part + row * D + d0;
      const f32x4 l0 = reinterpret_cast<const f32x4*>(src)[0], l1 = reinterpret_cast<const f32x4*>(src)[1];
      const f32x4 h0 = reinterpret_cast<const f32x4*>(src + D / 2)[0], h1 = reinterpret_cast<const f32x4*>(src + D / 2)[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x1[j] += l0[j];
        x1[4 + j] += l1[j];
        x2[j] += h0[j];
        x2[4 + j] += h1[j];
      }
    }
    if (which == 0 && (a.flags & PICO_ATTN_ROPE_BWD)) rope_bwd8(a, key, d0, x1, x2);
    u16x8 o1, o2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = f2bf(x1[j]);
      o2[j] = f2bf(x2[j]);
    }
    bf16_t* dst = which ? (bf16_t*)a.dv + b * a.dv_strides[0] + key * a.dv_strides[1] + hk * a.dv_strides[2]
                        : (bf16_t*)a.dk + b * a.dk_strides[0] + key * a.dk_strides[1] + hk * a.dk_strides[2];
    *reinterpret_cast<u16x8*>(dst + d0) = o1;
    *reinterpret_cast<u16x8*>(dst + d0 + D / 2) = o2;
  }
}

