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

// 8 fp32 accumulator registers -> bf16x8 MFMA operand fragment (round to nearest even).
PICO_DEV bf16x8 pack_frag(const float* v) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
  return r;
}

PICO_DEV float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
