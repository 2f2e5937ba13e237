// Probe: cycles per v_mfma_f32_32x32x16_bf16 whose A operand is a ds_read_b128 issued RD MFMAs earlier (a
// ring of RD + 1 operand registers), with F independent v_fma fillers per MFMA, at 1 or 2 waves per SIMD.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probes/mfma_lds_probe scripts/probes/mfma_lds_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

template <int N, int F, class T>
__device__ __forceinline__ void fillers(T& x, float c) {
#pragma unroll
  for (int k = 0; k < F; ++k) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x[k & 15]) : "v"(c));
}

template <int RD, int F, bool TR>
__global__ __launch_bounds__(256) void probe(float* out, unsigned long long* cyc, int iters, float c) {
  __shared__ __attribute__((aligned(16))) char smem[16384];
  for (int i = threadIdx.x; i < 4096; i += 256) ((float*)smem)[i] = 0.001f * i;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  bf16x8 b;
  for (int i = 0; i < 8; ++i) b[i] = (__bf16)(i * 0.5f);
  f32x16 acc = (f32x16)0.f;
  float x[16];
  for (int k = 0; k < 16; ++k) x[k] = threadIdx.x * 0.01f + k;
  const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem + ((lane * 16) & 4095);
  bf16x8 ring[RD + 1];
  auto rd = [&](int u) -> bf16x8 {
    bf16x8 v;
    if constexpr (TR) {
      typedef __attribute__((ext_vector_type(4))) short i16x4;
      i16x4 lo, hi;
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:0" : "=v"(lo) : "v"(base + (u & 3) * 1024));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:512" : "=v"(hi) : "v"(base + (u & 3) * 1024));
      v = __builtin_bit_cast(bf16x8, (__attribute__((ext_vector_type(8))) short){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
    } else {
      asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(v) : "v"(base + (u & 3) * 4096 % 16384));
    }
    return v;
  };
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int u = 0; u < RD; ++u) ring[u] = rd(u);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < RD + 1; ++u) {
      ring[(u + RD) % (RD + 1)] = rd(u);
      // wait until only the RD younger reads are outstanding (TR: two instructions per read)
      if constexpr (TR) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(2 * RD) : "memory");
      else asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(RD) : "memory");
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(ring[u]), "v"(b));
      fillers<16, F>(x, c);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int k = 0; k < 16; ++k) s += x[k];
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int RD, int F, bool TR>
void run(int blocks, int iters) {
  float* out; unsigned long long* cyc;
  (void)hipMalloc(&out, blocks * 256 * 4);
  (void)hipMalloc(&cyc, blocks * 4 * 8);
  probe<RD, F, TR><<<blocks, 256>>>(out, cyc, iters, 1.0001f);
  (void)hipDeviceSynchronize();
  probe<RD, F, TR><<<blocks, 256>>>(out, cyc, iters, 1.0001f);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 4);
  (void)hipMemcpy(h.data(), cyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
  double m = 0; for (auto v : h) m += v; m /= h.size();
  printf("{\"read\": \"%s\", \"rd\": %d, \"fillers\": %d, \"waves_per_simd\": %d, \"cyc_per_mfma\": %.2f}\n", TR ? "tr_b16x2" : "b128",
         RD, F, blocks / 256, m / (iters * (RD + 1.0)));
  (void)hipFree(out); (void)hipFree(cyc);
}

int main() {
  for (int w = 1; w <= 4; w *= 2) {
    const int bl = 256 * w;
    run<1, 0, false>(bl, 800); run<2, 0, false>(bl, 600); run<4, 0, false>(bl, 400); run<8, 0, false>(bl, 200);
    run<1, 5, false>(bl, 800); run<2, 5, false>(bl, 600); run<4, 5, false>(bl, 400); run<8, 5, false>(bl, 200);
    run<2, 0, true>(bl, 600); run<4, 0, true>(bl, 400); run<2, 5, true>(bl, 600); run<4, 5, true>(bl, 400);
  }
  return 0;
}
