// Probe: cycles per (1 v_mfma_f32_32x32x16_bf16 + K independent fillers) per wave, MFMA accumulator in
// VGPRs vs AGPRs, fillers v_fma_f32 or v_exp_f32, at 1 or 2 waves per SIMD. Build:
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mfma_valu_probe scripts/probes/mfma_valu_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

template <int K, bool AGPR, bool EXP>
__global__ __launch_bounds__(256) void probe(float* out, unsigned long long* cyc, int iters, float c) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(threadIdx.x * 0.001f + i); b[i] = (__bf16)(i * 0.5f); }
  f32x16 acc = (f32x16)0.f;
  float x[16];
  for (int k = 0; k < 16; ++k) x[k] = threadIdx.x * 0.01f + k;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if constexpr (AGPR) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
      else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if constexpr (EXP) asm volatile("v_exp_f32 %0, %0" : "+v"(x[(k + 4 * u) & 15]));
        else asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x[(k + 4 * u) & 15]) : "v"(c));
      }
    }
  }
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int k = 0; k < 16; ++k) s += x[k];
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int K, bool AGPR, bool EXP>
void run(const char* name, int blocks, int iters) {
  float* out; unsigned long long* cyc;
  hipMalloc(&out, blocks * 256 * 4);
  hipMalloc(&cyc, blocks * 4 * 8);
  probe<K, AGPR, EXP><<<blocks, 256>>>(out, cyc, iters, 1.0001f);
  hipDeviceSynchronize();
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  probe<K, AGPR, EXP><<<blocks, 256>>>(out, cyc, iters, 1.0001f);
  hipEventRecord(e1);
  hipDeviceSynchronize();
  float ms; hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(blocks * 4);
  hipMemcpy(h.data(), cyc, blocks * 4 * 8, hipMemcpyDeviceToHost);
  double m = 0; for (auto v : h) m += v; m /= h.size();
  printf("{\"probe\": \"%s\", \"fillers\": %d, \"agpr\": %d, \"exp\": %d, \"waves_per_simd\": %d, \"cyc_per_mfma\": %.2f, \"us\": %.1f}\n",
         name, K, AGPR, EXP, blocks / 256, m / (iters * 4.0), ms * 1e3);
  hipFree(out); hipFree(cyc);
}

int main() {
  const int it = 2000;
  for (int w = 1; w <= 2; ++w) {
    const int bl = 256 * w;
    run<0, false, false>("mfma_only", bl, it);
    run<0, true, false>("mfma_only", bl, it);
    run<4, false, false>("fma4", bl, it);
    run<4, true, false>("fma4", bl, it);
    run<6, false, false>("fma6", bl, it);
    run<6, true, false>("fma6", bl, it);
    run<8, false, false>("fma8", bl, it);
    run<8, true, false>("fma8", bl, it);
    run<12, false, false>("fma12", bl, it);
    run<12, true, false>("fma12", bl, it);
    run<2, false, true>("exp2", bl, it);
    run<2, true, true>("exp2", bl, it);
    run<4, false, true>("exp4", bl, it);
    run<4, true, true>("exp4", bl, it);
  }
  return 0;
}
