// AdamW step for gfx950 over every parameter of a model in ONE launch (HBM-bound).
//
// Replaces torch.optim.AdamW(model.parameters(), lr, fused=True).step() (ref train.py:13,204-209,235):
// ATen's fused AdamW walks the parameter list in multi_tensor_apply chunks (~60 launches per
// SmolLM-1.7B step at ~3.4 TB/s). Here a device table describes the tensors once (param, grad,
// exp_avg, exp_avg_sq pointers and sizes, all in the parameter dtype as torch keeps them), a chunk
// table maps workgroups to 64 Ki-element ranges, and each lane streams 8-element vectors.
// Per element, with ATen's fused AdamW expression types and order (fp32 values, double hyper-parameters,
// so the weight-decay and moment updates evaluate in double and round once to fp32; decoupled decay first):
//   p -= lr * wd * p;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g g;
//   p -= (float)(lr / bc1) * m / (float)(sqrt(v) / sqrt(bc2) + eps),  bc_i = 1 - b_i^step (host, double).
// Bytes per element: 8 read (p, g, m, v) + 6 written (p, m, v) for bf16 (10 read with an fp32 main_grad).
#include "common.h"

namespace {

constexpr int CHUNK = 65536;  // elements per workgroup

struct AdamHyper {
  double lr_wd, b1, b2, eps, bc2_sqrt;
  float step_size;
};

PICO_DEV void adam_elem(float& p, float g, float& m, float& v, const AdamHyper& h) {
  p -= h.lr_wd * p;
  m = h.b1 * m + (1 - h.b1) * g;
  v = h.b2 * v + (1 - h.b2) * g * g;
  const float denom = sqrtf(v) / h.bc2_sqrt + h.eps;
  p -= h.step_size * m / denom;
}

// tensors: [n_tensors][5] = (param, grad, exp_avg, exp_avg_sq pointers, grad_is_f32) as int64; sizes:
// [n_tensors] numel; chunks: [n_chunks][2] (tensor index, first element).
// grad_is_f32 = 1: the gradient is DataParallelBucket's averaged fp32 main_grad (its bf16 .grad cast
// deferred, ref picotron/data_parallel/data_parallel.py:165): each element is rounded to bf16 in register
// exactly as pico_cast_f32_bf16 would store it, so the step is bit-identical to cast-then-step, without the
// bf16 .grad write and re-read.
template <bool GF32>
PICO_DEV void load_grad8(const void* g, int64_t i, float (&out)[8]) {
  if constexpr (GF32) {
    const f32x4 a = reinterpret_cast<const f32x4*>((const float*)g + i)[0];
    const f32x4 b = reinterpret_cast<const f32x4*>((const float*)g + i)[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      out[j] = bf2f(f2bf(a[j]));
      out[4 + j] = bf2f(f2bf(b[j]));
    }
  } else {
    const u16x8 gv = *reinterpret_cast<const u16x8*>((const bf16_t*)g + i);
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = bf2f(gv[j]);
  }
}

template <bool GF32>
PICO_DEV void adamw_chunk(bf16_t* p, const void* g, bf16_t* m, bf16_t* v, int64_t n, int64_t c0, const AdamHyper& h) {
  const int64_t end = min(n, c0 + CHUNK);
  const bool vec = ((((uintptr_t)p | (uintptr_t)m | (uintptr_t)v) & 15) == 0) &&
                   (((uintptr_t)g & (GF32 ? 31 : 15)) == 0) && (n % 8 == 0);
  if (vec) {
    for (int64_t i = c0 + 8 * (int64_t)threadIdx.x; i < end; i += 8 * 256) {
      u16x8 pv = *reinterpret_cast<const u16x8*>(p + i);
      u16x8 mv = *reinterpret_cast<const u16x8*>(m + i), vv = *reinterpret_cast<const u16x8*>(v + i);
      float gf[8];
      load_grad8<GF32>(g, i, gf);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float pf = bf2f(pv[j]), mf = bf2f(mv[j]), vf = bf2f(vv[j]);
        adam_elem(pf, gf[j], mf, vf, h);
        pv[j] = f2bf(pf);
        mv[j] = f2bf(mf);
        vv[j] = f2bf(vf);
      }
      *reinterpret_cast<u16x8*>(p + i) = pv;
      *reinterpret_cast<u16x8*>(m + i) = mv;
      *reinterpret_cast<u16x8*>(v + i) = vv;
    }
  } else {
    for (int64_t i = c0 + threadIdx.x; i < end; i += 256) {
      float pf = bf2f(p[i]), mf = bf2f(m[i]), vf = bf2f(v[i]);
      const float gf = GF32 ? bf2f(f2bf(((const float*)g)[i])) : bf2f(((const bf16_t*)g)[i]);
      adam_elem(pf, gf, mf, vf, h);
      p[i] = f2bf(pf);
      m[i] = f2bf(mf);
      v[i] = f2bf(vf);
    }
  }
}

__global__ __launch_bounds__(256) void adamw_bf16_kernel(const int64_t* __restrict__ tensors,
                                                         const int64_t* __restrict__ sizes,
                                                         const int64_t* __restrict__ chunks, AdamHyper h) {
  const int64_t ti = chunks[2 * blockIdx.x], c0 = chunks[2 * blockIdx.x + 1];
  const int64_t* t = tensors + 5 * ti;
  bf16_t* p = (bf16_t*)t[0];
  const void* g = (const void*)t[1];
  bf16_t* m = (bf16_t*)t[2];
  bf16_t* v = (bf16_t*)t[3];
  if (t[4]) adamw_chunk<true>(p, g, m, v, sizes[ti], c0, h);
  else adamw_chunk<false>(p, g, m, v, sizes[ti], c0, h);
}

}  // namespace

extern "C" int64_t pico_adamw_chunk_elems(void) { return CHUNK; }

extern "C" int pico_adamw_bf16(const int64_t* tensors, const int64_t* sizes, const int64_t* chunks, int64_t n_chunks,
                               double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step,
                               void* stream) {
  PICO_REQUIRE(n_chunks >= 0 && n_chunks < (1ll << 31), "pico_adamw_bf16: bad chunk count");
  PICO_REQUIRE(step >= 1, "pico_adamw_bf16: step must be >= 1");
  PICO_REQUIRE(lr >= 0.0 && eps >= 0.0 && beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0,
               "pico_adamw_bf16: invalid hyper-parameters");
  if (n_chunks == 0) return 0;
  PICO_REQUIRE(tensors && sizes && chunks, "pico_adamw_bf16: null table");
  // bias corrections on the host in double, as ATen's fused AdamW takes them (then fp32 in the kernel)
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  AdamHyper h;
  h.lr_wd = (double)lr * (double)weight_decay;
  h.b1 = beta1;
  h.b2 = beta2;
  h.eps = eps;
  h.bc2_sqrt = sqrt(bc2);
  h.step_size = (float)((double)lr / bc1);
  hipStream_t s = (hipStream_t)stream;
  PICO_TRY(pico_launch(PICO_K_ADAMW, "adamw", adamw_bf16_kernel, dim3((int)n_chunks), dim3(256), 0, s, tensors, sizes, chunks, h));
  return 0;
}
