// Fused AdamW over the flat parameter arena (K8 in SURVEY.md §2.11).
//
// One pass over numel elements: reads the fp32 (default) or bf16 grad, fp32 master/exp_avg/exp_avg_sq
// and a per-2048-element-chunk weight-decay flag; writes master/m/v and the bf16
// compute copy.  Hyper-parameters (lr, betas, eps, wd, bias corrections, clip)
// and the global gradient sum-of-squares are read from DEVICE memory, so a
// captured HIP graph replays correct steps without host round trips.
// 26 bytes/element of HBM traffic: the 124M-parameter step is ~3.2 GB, ~0.6 ms.
#include <cstdlib>
#include "common.h"

// non-temporal loads / stores for the once-per-step streams (A/B builds: -DADAMW_NT=0/1)
#ifndef ADAMW_NT
#define ADAMW_NT 1  // Llama-7B step: AdamW 33.6 vs 34.3 ms, grad norm 4.32 vs 4.44 (profiles/ab/adamw_nt_r04.log)
#endif

namespace orion {

template <typename T>
ORION_DEVICE T ld_stream(const T* p) {
  if constexpr (ADAMW_NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <typename T>
ORION_DEVICE void st_stream(T v, T* p) {
  if constexpr (ADAMW_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

constexpr int ADAM_CHUNK = 2048;  // must match orion_amd/train/flat.py ALIGN

// 8 consecutive gradient elements as fp32 (arena in fp32 or bf16)
ORION_DEVICE void load8(const float* g, long e, float (&f)[8]) {
  const f32x4 a = ld_stream(reinterpret_cast<const f32x4*>(g + e)), b = ld_stream(reinterpret_cast<const f32x4*>(g + e + 4));
#pragma unroll
  for (int j = 0; j < 4; ++j) { f[j] = a[j]; f[4 + j] = b[j]; }
}
ORION_DEVICE void load8(const bf16_t* g, long e, float (&f)[8]) {
  const bf16x8 v = ld_stream(reinterpret_cast<const bf16x8*>(g + e));
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = bf2f(v[j]);
}
ORION_DEVICE void load4(const float* g, long e, float (&f)[4]) {
  const f32x4 a = ld_stream(reinterpret_cast<const f32x4*>(g + e));
#pragma unroll
  for (int j = 0; j < 4; ++j) f[j] = a[j];
}
ORION_DEVICE void load4(const bf16_t* g, long e, float (&f)[4]) {
  const bf16x4 v = ld_stream(reinterpret_cast<const bf16x4*>(g + e));
#pragma unroll
  for (int j = 0; j < 4; ++j) f[j] = bf2f(v[j]);
}

// partial[b] = sum of squares over this workgroup's grid-stride slice
template <typename G>
__global__ __launch_bounds__(256) void sumsq_partial_kernel(const G* __restrict__ g, long n8,
                                                            float* __restrict__ partial) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8];
    load8(g, i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j] * v[j];
  }
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(1024) void sum_partials_kernel(const float* __restrict__ partial,
                                                            int P, float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < P; i += 1024) s += partial[i];
  s = block_sum<16>(s, red);
  if (threadIdx.x == 0) out[0] = s;
}

#ifndef ADAMW_UNROLL
#define ADAMW_UNROLL 2
#endif

// hyper = [lr, beta1, beta2, eps, weight_decay, 1-beta1^t, 1-beta2^t, max_grad_norm]
template <typename G>
__global__ __launch_bounds__(256) void adamw_flat_kernel(
    bf16_t* __restrict__ p16, float* __restrict__ master, float* __restrict__ m,
    float* __restrict__ v, const G* __restrict__ g, const uint8_t* __restrict__ decay,
    const float* __restrict__ hyper, const float* __restrict__ sumsq, long n4) {
  const float lr = hyper[0], b1 = hyper[1], b2 = hyper[2], eps = hyper[3], wd = hyper[4];
  const float bc1 = hyper[5], bc2 = hyper[6], clip = hyper[7];
  float cs = 1.f;
  if (clip > 0.f) {
    const float norm = sqrtf(sumsq[0]);
    cs = fminf(1.f, clip / (norm + 1e-6f));
  }
  const float step = lr / bc1;
  const float inv_bc2 = 1.f / bc2;
  // ADAMW_UNROLL groups of 4 elements per thread and iteration, every load of the iteration
  // issued before the first update (more bytes in flight per thread; same per-element math)
  const long stride = (long)gridDim.x * 256;
  for (long i0 = blockIdx.x * 256L + threadIdx.x; i0 < n4; i0 += ADAMW_UNROLL * stride) {
    f32x4 w[ADAMW_UNROLL], mm[ADAMW_UNROLL], vv[ADAMW_UNROLL];
    float gg[ADAMW_UNROLL][4];
    float dec[ADAMW_UNROLL];
#pragma unroll
    for (int u = 0; u < ADAMW_UNROLL; ++u) {
      const long i = i0 + u * stride;
      if (u == 0 || i < n4) {
        const long e = i * 4;
        dec[u] = decay[e / ADAM_CHUNK] ? (1.f - lr * wd) : 1.f;
        w[u] = ld_stream(reinterpret_cast<const f32x4*>(master + e));
        mm[u] = ld_stream(reinterpret_cast<const f32x4*>(m + e));
        vv[u] = ld_stream(reinterpret_cast<const f32x4*>(v + e));
        load4(g, e, gg[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < ADAMW_UNROLL; ++u) {
      const long i = i0 + u * stride;
      if (u > 0 && i >= n4) break;
      const long e = i * 4;
      bf16x4 out;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // every multiply-add an explicit fmaf: left to the compiler's contraction, the two
        // unrolled copies fused differently (1-ulp differences between elements handled by
        // slot 0 and slot 1, i.e. results depending on the grid: tests/test_grid_forms_gpu.py)
        const float gr = gg[u][j] * cs;
        mm[u][j] = fmaf(b1, mm[u][j], (1.f - b1) * gr);
        vv[u][j] = fmaf(b2, vv[u][j], ((1.f - b2) * gr) * gr);
        const float denom = sqrtf(vv[u][j] * inv_bc2) + eps;
        w[u][j] = fmaf(w[u][j], dec[u], -(step * mm[u][j] / denom));
        out[j] = f2bf(w[u][j]);
      }
      st_stream(w[u], reinterpret_cast<f32x4*>(master + e));
      st_stream(mm[u], reinterpret_cast<f32x4*>(m + e));
      st_stream(vv[u], reinterpret_cast<f32x4*>(v + e));
      st_stream(out, reinterpret_cast<bf16x4*>(p16 + e));
    }
  }
}

}  // namespace orion

using namespace orion;

constexpr int SUMSQ_BLOCKS = 1024;

int orion_sumsq_partials() { return SUMSQ_BLOCKS; }

// out[0] = sum(g^2) over an fp32 (g_f32) or bf16 arena; partial holds SUMSQ_BLOCKS floats.
int orion_grad_sumsq(const void* g, long n, int g_f32, float* partial, float* out, hipStream_t st) {
  if (n % 8) return -1;
  if (g_f32) sumsq_partial_kernel<float><<<SUMSQ_BLOCKS, 256, 0, st>>>((const float*)g, n / 8, partial);
  else sumsq_partial_kernel<bf16_t><<<SUMSQ_BLOCKS, 256, 0, st>>>((const bf16_t*)g, n / 8, partial);
  sum_partials_kernel<<<1, 1024, 0, st>>>(partial, SUMSQ_BLOCKS, out);
  return (int)hipGetLastError();
}

int orion_adamw_flat(void* p16, float* master, float* m, float* v, const void* g, int g_f32,
                     const uint8_t* decay, const float* hyper, const float* sumsq, long n,
                     hipStream_t st) {
  if (n % ADAM_CHUNK) return -1;
  const long n4 = n / 4;
  // One 4-element group per thread (the loop only runs past 2^22 workgroups): on MI355X the
  // one-shot grid streams at 5.8-6.1 TB/s over GPT-2's arena against 4.4-4.6 for a 4,096-
  // workgroup grid-stride loop (0.61-0.64 vs 0.82-0.86 ms; 1 G parameters 5.03 vs 5.68 ms;
  // profiles/ab/adamw_grid_r05.log).  ORION_ADAMW_GRID (diagnostic) caps the grid.
  static const long cap = [] {
    const char* e = getenv("ORION_ADAMW_GRID");
    const long c = e ? atol(e) : 0;
    return c > 0 ? c : (1L << 22);
  }();
  long grid = (n4 + 255) / 256;
  if (grid > cap) grid = cap;
  if (g_f32)
    adamw_flat_kernel<float><<<(int)grid, 256, 0, st>>>((bf16_t*)p16, master, m, v, (const float*)g,
                                                        decay, hyper, sumsq, n4);
  else
    adamw_flat_kernel<bf16_t><<<(int)grid, 256, 0, st>>>((bf16_t*)p16, master, m, v,
                                                         (const bf16_t*)g, decay, hyper, sumsq, n4);
  return (int)hipGetLastError();
}
