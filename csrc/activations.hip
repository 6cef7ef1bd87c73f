// Elementwise activations (K4 GELU-tanh + bias, K7 SwiGLU) and small helpers.
//
// All are HBM-bound: 16-byte vector loads/stores of 8 bf16 per lane, fp32
// math.  The GELU backward fuses the bias-gradient column sum: each lane owns
// 8 fixed columns for every row its workgroup visits, so dbias partials stay in
// registers (no second pass over the (rows, 4C) activation).
#include <cstdlib>
#include "common.h"

namespace orion {

ORION_DEVICE void ld8(const bf16_t* p, float* o) {
  bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = bf2f(v[j]);
}
ORION_DEVICE void st8(bf16_t* p, const float* o) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(o[j]);
  *reinterpret_cast<bf16x8*>(p) = v;
}

// y = gelu(x + b); rows x C, C % 8 == 0.  Grid-stride over 8-element chunks.
__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ b, bf16_t* __restrict__ y,
    long n8, int C8) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8], bb[8];
    ld8(x + i * 8, v);
    if (b) ld8(b + (i % C8) * 8, bb);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_tanh_f(v[j] + (b ? bb[j] : 0.f));
    st8(y + i * 8, v);
  }
}

// dx = dy * gelu'(x + b); part_db[blk][c] = sum over this block's rows of dx.
// grid = (row_blocks, ceil(C/512)); block = 4 waves, lane owns 8 columns.
__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ b,
    bf16_t* __restrict__ dx, float* __restrict__ part_db, int rows, int C, int rows_per_block) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = (blockIdx.y * 64 + lane) * 8;
  const bool valid = c < C;
  float bb[8], acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { bb[j] = 0.f; acc[j] = 0.f; }
  if (valid && b) ld8(b + c, bb);
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = valid ? min(rows, r0 + rows_per_block) : 0;
  for (int r = r0 + wv; r < r1; r += 4) {
    float xv[8], g[8];
    ld8(x + (size_t)r * C + c, xv);
    ld8(dy + (size_t)r * C + c, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      g[j] *= gelu_tanh_grad_f(xv[j] + bb[j]);
      acc[j] += g[j];
    }
    st8(dx + (size_t)r * C + c, g);
  }
  if (!part_db) return;  // uniform across the block
  __shared__ float red[4][512];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[wv][lane * 8 + j] = acc[j];
  __syncthreads();
  if (wv == 0 && valid) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = lane * 8 + j;
      part_db[(size_t)blockIdx.x * C + c + j] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
    }
  }
}

// SwiGLU on a packed [rows][2F] projection (gate | up) -> [rows][F].
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(
    const bf16_t* __restrict__ gu, bf16_t* __restrict__ y, long n8, int F8) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long r = i / F8, c = i % F8;
    const bf16_t* base = gu + r * (2L * F8 * 8);
    float g[8], u[8];
    ld8(base + c * 8, g);
    ld8(base + (F8 + c) * 8, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = silu_f(g[j]) * u[j];
    st8(y + i * 8, g);
  }
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ gu, bf16_t* __restrict__ dgu,
    long n8, int F8) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long r = i / F8, c = i % F8;
    const long off = r * (2L * F8 * 8);
    float g[8], u[8], d[8], dg[8], du[8];
    ld8(gu + off + c * 8, g);
    ld8(gu + off + (F8 + c) * 8, u);
    ld8(dy + i * 8, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float s = 1.f / (1.f + __expf(-g[j]));
      const float sl = g[j] * s;
      du[j] = d[j] * sl;
      dg[j] = d[j] * u[j] * (s + sl * (1.f - s));
    }
    st8(dgu + off + c * 8, dg);
    st8(dgu + off + (F8 + c) * 8, du);
  }
}

// x *= (*scale) for bf16 x (scale lives on the device: no host sync).
__global__ __launch_bounds__(256) void scale_bf16_kernel(bf16_t* __restrict__ x,
                                                         const float* __restrict__ scale,
                                                         long n8) {
  const float s = *scale;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8];
    ld8(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] *= s;
    st8(x + i * 8, v);
  }
}

// out[i] = (*scale) * sum_s slabs[s][i] (+ out[i] when accumulating): the combine step of
// the split-K weight gradient (S fp32 slabs from one launch over token chunks), with the
// LM head's 1/n_valid * upstream-grad scale folded in.  out is the parameter's slice of
// the gradient arena, fp32 (f32 != 0) or bf16.  Fixed summation order: deterministic.
#ifndef SLAB_NT
#define SLAB_NT 1  // 13.65 vs 14.1 us per call in the GPT-2 step (profiles/ab/slab_rmsdres_nt_r04.log)
#endif
// the slabs are read once, right after the weight-gradient kernel wrote them
ORION_DEVICE f32x4 ld_slab(const f32x4* p) {
  if constexpr (SLAB_NT) return __builtin_nontemporal_load(p);
  else return *p;
}

__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ slabs, int S,
                                                       long n4, void* __restrict__ out,
                                                       const float* __restrict__ scale,
                                                       int accumulate, int f32) {
  const float sc = scale ? *scale : 1.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    // slabs in fixed order 0, 1, ..., S - 1 (deterministic), loaded 8 at a time (measured
    // 14.1 vs 14.7 us per call: the sums are bound by the ~66 MB of slabs each reads,
    // profiles/ab/slab_sum_unroll_r04.log)
    const f32x4* sp = reinterpret_cast<const f32x4*>(slabs) + i;
    const long sstride = n4;
    f32x4 acc = ld_slab(sp);
    for (int k = 1; k < S; k += 8) {  // S is uniform: the guards are scalar branches
      f32x4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k + u < S) t[u] = ld_slab(sp + (k + u) * sstride);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k + u < S) acc += t[u];
    }
    acc *= sc;
    if (f32) {
      f32x4* o = reinterpret_cast<f32x4*>(out) + i;
      *o = accumulate ? *o + acc : acc;
    } else {
      bf16x4* o = reinterpret_cast<bf16x4*>(out) + i;
      bf16x4 r;
      if (accumulate) {
        const bf16x4 prev = *o;
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = f2bf(acc[j] + bf2f(prev[j]));
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) r[j] = f2bf(acc[j]);
      }
      *o = r;
    }
  }
}

}  // namespace orion

using namespace orion;

static inline int ew_grid(long n8) {
  // One group per thread (the grid-stride loop only runs past 2^22 workgroups): swiglu_fwd
  // over Llama's gate|up 0.218 -> 0.191 ms against a 2,048-workgroup loop, as for AdamW
  // (profiles/ab/ew_grid_r05.log).  ORION_EW_GRID (diagnostic) caps the grid.
  static const long cap = [] {
    const char* e = getenv("ORION_EW_GRID");
    const long c = e ? atol(e) : 0;
    return c > 0 ? c : (1L << 22);
  }();
  long g = (n8 + 255) / 256;
  return (int)(g < cap ? (g < 1 ? 1 : g) : cap);
}

int orion_layernorm_bwd_blocks(int rows);

int orion_bias_gelu_fwd(const void* x, const void* b, void* y, long n, int C, hipStream_t st) {
  if (C % 8 || n % 8) return -1;
  const long n8 = n / 8;
  bias_gelu_fwd_kernel<<<ew_grid(n8), 256, 0, st>>>((const bf16_t*)x, (const bf16_t*)b,
                                                    (bf16_t*)y, n8, C / 8);
  return (int)hipGetLastError();
}

int orion_bias_gelu_bwd(const void* dy, const void* x, const void* b, void* dx, float* part,
                        int rows, int C, hipStream_t st) {
  if (C % 8) return -1;
  const int nb = orion_layernorm_bwd_blocks(rows);
  const int rpb = (rows + nb - 1) / nb;
  dim3 grid(nb, (C / 8 + 63) / 64);
  bias_gelu_bwd_kernel<<<grid, 256, 0, st>>>((const bf16_t*)dy, (const bf16_t*)x,
                                             (const bf16_t*)b, (bf16_t*)dx, part, rows, C, rpb);
  return (int)hipGetLastError();
}

int orion_swiglu_fwd(const void* gu, void* y, long rows, int F, hipStream_t st) {
  if (F % 8) return -1;
  const long n8 = rows * (F / 8);
  swiglu_fwd_kernel<<<ew_grid(n8), 256, 0, st>>>((const bf16_t*)gu, (bf16_t*)y, n8, F / 8);
  return (int)hipGetLastError();
}

int orion_swiglu_bwd(const void* dy, const void* gu, void* dgu, long rows, int F, hipStream_t st) {
  if (F % 8) return -1;
  const long n8 = rows * (F / 8);
  swiglu_bwd_kernel<<<ew_grid(n8), 256, 0, st>>>((const bf16_t*)dy, (const bf16_t*)gu,
                                                 (bf16_t*)dgu, n8, F / 8);
  return (int)hipGetLastError();
}

int orion_scale_bf16(void* x, const float* scale, long n, hipStream_t st) {
  if (n % 8) return -1;
  const long n8 = n / 8;
  scale_bf16_kernel<<<ew_grid(n8), 256, 0, st>>>((bf16_t*)x, scale, n8);
  return (int)hipGetLastError();
}

int orion_slab_sum(const float* slabs, int S, long n, void* out, const float* scale,
                   int accumulate, int out_f32, hipStream_t st) {
  if (n % 4) return -1;
  const long n4 = n / 4;
  slab_sum_kernel<<<ew_grid(n4 / 2), 256, 0, st>>>(slabs, S, n4, out, scale, accumulate, out_f32);
  return (int)hipGetLastError();
}
