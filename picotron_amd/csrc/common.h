// Shared helpers for the picotron_amd gfx950 kernels.
// All kernels are bf16-in/bf16-out with fp32 arithmetic; every entry point takes the
// caller's hipStream_t and never allocates (workspaces come from the caller).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include "../../include/picotron_hip.h"

typedef uint16_t bf16_t;  // raw bf16 bits on the host/kernel ABI
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4;
typedef __attribute__((ext_vector_type(2))) unsigned short u16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short i16x4;

#define PICO_DEV __device__ __forceinline__

PICO_DEV float bf2f(unsigned short u) { return __uint_as_float(((unsigned)u) << 16); }

// Round-to-nearest-even f32 -> bf16 (hipcc lowers the cast to v_cvt_pk_bf16_f32 on gfx950,
// which keeps NaN a NaN: MI355X_MICROARCH.md "Correctness boundaries").
PICO_DEV unsigned short f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}

PICO_DEV unsigned pack2bf(float lo, float hi) {
  return (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
}

// ---------------------------------------------------------------------------------------
// Host-side status / profiling plumbing (defined in runtime.cpp)
// ---------------------------------------------------------------------------------------
int pico_set_error(const char* fmt, ...);
int pico_check_launch(const char* op);
void pico_prof_pre(int kid, hipStream_t s);
void pico_prof_post(int kid, hipStream_t s);

#define PICO_REQUIRE(cond, ...)               \
  do {                                        \
    if (!(cond)) return pico_set_error(__VA_ARGS__); \
  } while (0)

// Launch wrapper: optional event timing of one kernel id, then error check.
#define PICO_LAUNCH(kid, opname, stream, ...)          \
  do {                                                 \
    pico_prof_pre((kid), (stream));                    \
    __VA_ARGS__;                                       \
    pico_prof_post((kid), (stream));                   \
    int _rc = pico_check_launch(opname);               \
    if (_rc) return _rc;                               \
  } while (0)

// Compile-time loop: f(std::integral_constant<int, I>{}) for I = 0 .. N-1.
template <int N, int I = 0, class F>
__host__ __device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

static inline int pico_cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
