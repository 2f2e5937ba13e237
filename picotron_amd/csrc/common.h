// Shared helpers for the picotron_amd gfx950 kernels.
// All kernels are bf16-in/bf16-out with fp32 arithmetic; every entry point takes the
// caller's hipStream_t and never allocates (workspaces come from the caller).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
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
// Host-side status / profiling plumbing (defined in runtime.hip)
// ---------------------------------------------------------------------------------------
int pico_set_error(const char* fmt, ...);
int pico_check_launch(const char* op);
// current value of a kernel-selection knob (PICO_SEL_*, pico_select; PICO_SEL_AUTO = the shape rule)
int pico_sel(int knob);
// true when kernel id `kid` is being timed: *start / *stop are the next free event pair of its pool
bool pico_prof_events(int kid, hipEvent_t* start, hipEvent_t* stop);

#define PICO_REQUIRE(cond, ...)               \
  do {                                        \
    if (!(cond)) return pico_set_error(__VA_ARGS__); \
  } while (0)

#define PICO_TRY(expr)         \
  do {                         \
    const int _rc = (expr);    \
    if (_rc) return _rc;       \
  } while (0)

// Every kernel launch of the library: the arguments are converted to the kernel's parameter types; while
// kernel id `kid` is timed (pico_prof_enable) the launch carries its own start / stop events
// (hipExtLaunchKernel: the dispatch packet's timestamps, i.e. the kernel's execution time as rocprofv3
// reports it, without the queue gap a pair of stream-recorded events would add); then the error check.
template <typename... KP, typename... Args>
int pico_launch(int kid, const char* op, void (*kernel)(KP...), dim3 grid, dim3 block, unsigned shmem, hipStream_t s,
                Args&&... args) {
  static_assert(sizeof...(KP) == sizeof...(Args), "pico_launch: argument count");
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (pico_prof_events(kid, &e0, &e1)) {
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, e0, e1, 0u, static_cast<KP>(args)...);
  } else {
    kernel<<<grid, block, shmem, s>>>(static_cast<KP>(args)...);
  }
  return pico_check_launch(op);
}

// Sum over the 64 lanes of a wave, result in every lane, without LDS (ds_bpermute) round trips:
// DPP within rows of 16 (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror), then
// v_permlane16_swap (row pairs) and v_permlane32_swap (halves).
PICO_DEV float wave_sum_dpp(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
  const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
}

// Compile-time loop: f(std::integral_constant<int, I>{}) for I = 0 .. N-1.
template <int N, int I = 0, class F>
__host__ __device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

static inline int pico_cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// compute units of the current device (cached per device; 256 on MI355X)
static inline int pico_num_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}
