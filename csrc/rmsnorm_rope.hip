// RMSNorm fwd/bwd (K5) and rotary position embedding fwd/bwd (K6) for the
// Llama family.
//
// RMSNorm: d_model is large (4096 for Llama-2-7B), so one 256-thread
// workgroup per row with 16-byte vectors (16 elements per lane at 4096); a
// fixed grid strides over rows so every thread owns the same column slices in
// every row and accumulates dgamma in registers (partials folded by a second
// kernel, deterministic).
// RoPE: rotate-half convention (x1, x2) -> (x1 cos - x2 sin, x2 cos + x1 sin)
// on a strided (B, T, H, D) view (e.g. the q or k slice of a packed QKV
// projection), output contiguous; cos/sin come from a host-built fp32 table
// (T, D/2) -- no device transcendental per element (HIP guide Appendix B).
#include "common.h"

// RMS_NT: the backward loads its saved input (read once, long after it was written) with the
// non-temporal hint: rms_bwd 89.3 vs 93.8 us at Llama-7B shapes; the same on the forward's
// residual stream measured neutral (profiles/ab/rms_nt_r04.log)
#ifndef RMS_DRES_NT
#define RMS_DRES_NT 1  // and the incoming residual gradient: rms_bwd 88.3 vs 89.4 us (profiles/ab/slab_rmsdres_nt_r04.log)
#endif
#ifndef RMS_NT
#define RMS_NT 1
#endif

namespace orion {

template <bool NT = false>
ORION_DEVICE void ld8f(const bf16_t* p, float* o) {
  bf16x8 v;
  if constexpr (NT && RMS_NT) v = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(p));
  else v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = bf2f(v[j]);
}
template <bool NT = false>
ORION_DEVICE void st8f(bf16_t* p, const float* o) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(o[j]);
  if constexpr (NT && RMS_NT) __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(p));
  else *reinterpret_cast<bf16x8*>(p) = v;
}

template <int IT>
__global__ __launch_bounds__(256) void rms_fwd_kernel(const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ w,
                                                      bf16_t* __restrict__ y,
                                                      float* __restrict__ rstd_out, int rows,
                                                      int C, float eps,
                                                      const bf16_t* __restrict__ res,
                                                      bf16_t* __restrict__ sum_out) {
  __shared__ float red[4];
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const bf16_t* xr = x + (size_t)row * C;
    float v[IT][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int c = (i * 256 + threadIdx.x) * 8;
      if (c < C) {
        ld8f(xr + c, v[i]);
        if (res) {  // fused residual add: s = x + r returned and normalised
          float rv[8];
          ld8f(res + (size_t)row * C + c, rv);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[i][j] = bf2f(f2bf(v[i][j] + rv[j]));
          st8f(sum_out + (size_t)row * C + c, v[i]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[i][j] * v[i][j];
      }
    }
    const float rstd = rsqrtf(block_sum<4>(s, red) / (float)C + eps);
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int c = (i * 256 + threadIdx.x) * 8;
      if (c < C) {
        float wf[8], o[8];
        ld8f(w + c, wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[i][j] * rstd * wf[j];
        st8f(y + (size_t)row * C + c, o);
      }
    }
    if (threadIdx.x == 0) rstd_out[row] = rstd;
  }
}

template <int IT>
__global__ __launch_bounds__(256) void rms_bwd_kernel(const bf16_t* __restrict__ dy,
                                                      const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ w,
                                                      const float* __restrict__ rstd_in,
                                                      bf16_t* __restrict__ dx,
                                                      float* __restrict__ part, int rows, int C,
                                                      const bf16_t* __restrict__ dres) {
  __shared__ float red[4];
  float wf[IT][8], adw[IT][8];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int c = (i * 256 + threadIdx.x) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) { wf[i][j] = 0.f; adw[i][j] = 0.f; }
    if (c < C) ld8f(w + c, wf[i]);
  }
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const float rstd = rstd_in[row];
    float xh[IT][8], g[IT][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int c = (i * 256 + threadIdx.x) * 8;
      if (c < C) {
        float xv[8], dv[8];
        ld8f<true>(x + (size_t)row * C + c, xv);
        ld8f(dy + (size_t)row * C + c, dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[i][j] = xv[j] * rstd;
          g[i][j] = dv[j] * wf[i][j];
          s += g[i][j] * xh[i][j];
          adw[i][j] += dv[j] * xh[i][j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { xh[i][j] = 0.f; g[i][j] = 0.f; }
      }
    }
    const float m = block_sum<4>(s, red) / (float)C;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int c = (i * 256 + threadIdx.x) * 8;
      if (c < C) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (g[i][j] - xh[i][j] * m);
        if (dres) {
          float rv[8];
          if constexpr (RMS_DRES_NT) ld8f<true>(dres + (size_t)row * C + c, rv);
          else ld8f(dres + (size_t)row * C + c, rv);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += rv[j];
        }
        st8f(dx + (size_t)row * C + c, o);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int c = (i * 256 + threadIdx.x) * 8;
    if (c < C) {
#pragma unroll
      for (int j = 0; j < 8; ++j) part[(size_t)blockIdx.x * C + c + j] = adw[i][j];
    }
  }
}

// out[b,t,h,:] = rope(x[b,t,h,:]); sign = +1 forward, -1 backward (inverse rotation).
// One thread per 8 rotation pairs.
// y may alias x (in-place backward on a strided gradient view): every thread reads its
// 16 elements before writing them and no two threads touch the same element.
__global__ __launch_bounds__(256) void rope_kernel(const bf16_t* x, long xsb, long xst, long xsh,
                                                   bf16_t* y, long ysb, long yst, long ysh,
                                                   const float* __restrict__ cosv,
                                                   const float* __restrict__ sinv, int B, int T,
                                                   int H, int D, int pos0, float sign) {
  const int P8 = D / 16;  // groups of 8 pairs per head
  const long n = (long)B * T * H * P8;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int pg = i % P8;
    const long row = i / P8;
    const int h = row % H;
    const long t = (row / H) % T;
    const long b = row / ((long)H * T);
    const bf16_t* xp = x + b * xsb + t * xst + h * xsh;
    bf16_t* yp = y + b * ysb + t * yst + h * ysh;
    float x1[8], x2[8], o1[8], o2[8];
    ld8f(xp + pg * 8, x1);
    ld8f(xp + D / 2 + pg * 8, x2);
    const float* cr = cosv + (t + pos0) * (long)(D / 2) + pg * 8;
    const float* sr = sinv + (t + pos0) * (long)(D / 2) + pg * 8;
    const f32x4 c0 = *reinterpret_cast<const f32x4*>(cr), c1 = *reinterpret_cast<const f32x4*>(cr + 4);
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(sr), s1 = *reinterpret_cast<const f32x4*>(sr + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float cc = j < 4 ? c0[j] : c1[j - 4];
      const float ss = (j < 4 ? s0[j] : s1[j - 4]) * sign;
      o1[j] = x1[j] * cc - x2[j] * ss;
      o2[j] = x2[j] * cc + x1[j] * ss;
    }
    st8f(yp + pg * 8, o1);
    st8f(yp + D / 2 + pg * 8, o2);
  }
}

}  // namespace orion

using namespace orion;

int orion_colsum_partials2(const float* part, float* mid, void* out, int P, int C, int f32,
                           hipStream_t st);

static int rms_blocks(int rows) { return rows < 1024 ? rows : 1024; }

int orion_rmsnorm_fwd(const void* x, const void* w, void* y, float* rstd, int rows, int C,
                      float eps, const void* res, void* sum_out, hipStream_t st) {
  if (C % 8) return -1;
  const int it = (C / 8 + 255) / 256;
  const int g = rows < 4096 ? rows : 4096;
  auto X = (const bf16_t*)x; auto W = (const bf16_t*)w; auto Y = (bf16_t*)y;
  auto R = (const bf16_t*)res; auto S = (bf16_t*)sum_out;
  switch (it) {
#define RF(K) case K: rms_fwd_kernel<K><<<g, 256, 0, st>>>(X, W, Y, rstd, rows, C, eps, R, S); break;
    RF(1) RF(2) RF(3) RF(4) RF(5) RF(6) RF(7) RF(8)
#undef RF
    default: return -2;
  }
  return (int)hipGetLastError();
}

int orion_rmsnorm_bwd_blocks(int rows) { return rms_blocks(rows); }

int orion_rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd, void* dx,
                      void* dw, float* part, int rows, int C, const void* dres, int dw_f32,
                      hipStream_t st) {
  if (C % 8) return -1;
  const int it = (C / 8 + 255) / 256;
  const int nb = rms_blocks(rows);
  auto DY = (const bf16_t*)dy; auto X = (const bf16_t*)x; auto W = (const bf16_t*)w;
  auto DX = (bf16_t*)dx;
  auto DR = (const bf16_t*)dres;
  switch (it) {
#define RB(K) case K: rms_bwd_kernel<K><<<nb, 256, 0, st>>>(DY, X, W, rstd, DX, part, rows, C, DR); break;
    RB(1) RB(2) RB(3) RB(4) RB(5) RB(6) RB(7) RB(8)
#undef RB
    default: return -2;
  }
  if (dw) return orion_colsum_partials2(part, part + (size_t)nb * C, dw, nb, C, dw_f32, st);
  return (int)hipGetLastError();
}

int orion_rope(const void* x, long xsb, long xst, long xsh, void* y, long ysb, long yst,
               long ysh, const float* cosv, const float* sinv, int B, int T, int H, int D,
               int pos0, float sign, hipStream_t st) {
  if (D % 16) return -1;
  if (!cosv || !sinv || !x || !y) return -3;
  const long n = (long)B * T * H * (D / 16);
  long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  rope_kernel<<<(int)g, 256, 0, st>>>((const bf16_t*)x, xsb, xst, xsh, (bf16_t*)y, ysb, yst, ysh,
                                      cosv, sinv, B, T, H, D, pos0, sign);
  return (int)hipGetLastError();
}
