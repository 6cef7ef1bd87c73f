// Shared device helpers for the orion_amd gfx950 (CDNA4, MI355X) kernels.
//
// Conventions used by every kernel in this directory:
//   * wave64 everywhere: lane = threadIdx.x & 63, reductions span 64 lanes;
//   * bf16 tensors are moved as 8- or 16-byte vectors (Guideline 13 of the
//     CDNA HIP guide: scalar bf16 loads cost ~2x);
//   * all arithmetic in fp32, bf16 conversion with round-to-nearest-even that
//     keeps NaN a NaN (plain cast -> v_cvt_pk_bf16_f32 at -O3).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define ORION_DEVICE __device__ __forceinline__

// Device-side bounds checks, compiled in only by the debug build (ORION_AMD_DEBUG=1,
// orion_amd/build.py): a failing check prints the kernel, line and condition and traps.
#ifdef ORION_DEBUG
#include <assert.h>
#define ORION_DASSERT(cond) assert(cond)
#else
#define ORION_DASSERT(cond) ((void)0)
#endif

namespace orion {

typedef unsigned short bf16_t;  // raw bf16 bits

typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) long i64x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned short bf16x4;
typedef __attribute__((ext_vector_type(8))) unsigned short bf16x8;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_mfma;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_mfma;

ORION_DEVICE float bf2f(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}

ORION_DEVICE bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(bf16_t, b);
}

ORION_DEVICE unsigned pack_bf16x2(float lo, float hi) {
  return (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
}

// Gradient-arena element I/O: the arena is fp32 by default (accumulation over micro-batches
// and the data-parallel reduction stay in fp32) or bf16 (opt-in); kernels that write a
// parameter's gradient slice take `void*` + a wave-uniform `f32` flag.
ORION_DEVICE void store_grad(void* p, long i, float v, int f32) {
  if (f32) static_cast<float*>(p)[i] = v;
  else static_cast<bf16_t*>(p)[i] = f2bf(v);
}

ORION_DEVICE float load_grad(const void* p, long i, int f32) {
  return f32 ? static_cast<const float*>(p)[i] : bf2f(static_cast<const bf16_t*>(p)[i]);
}

template <int N>
struct VecT;
template <>
struct VecT<4> { typedef bf16x4 type; };
template <>
struct VecT<8> { typedef bf16x8 type; };

// ---------------------------------------------------------------- wave / block reductions
ORION_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

ORION_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x = 64 * NW; `scratch` holds NW floats in LDS.
template <int NW>
ORION_DEVICE float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) r += scratch[i];
  __syncthreads();
  return r;
}

template <int NW>
ORION_DEVICE float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max(v);
  if (lane == 0) scratch[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NW; ++i) r = fmaxf(r, scratch[i]);
  __syncthreads();
  return r;
}

// GELU (tanh approximation) and its derivative, as in GPT-2 / nanoGPT.
// 0.5 (1 + tanh(u)) == sigmoid(2u) = 1 / (1 + 2^(-2u log2 e)): one v_exp_f32 + one v_rcp_f32
// instead of a tanhf expansion (the activation kernels are HBM-bound only if the VALU keeps up).
ORION_DEVICE float sigmoid2u_(float x, float* x2out) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float m2log2e = -2.8853900817779268f;  // -2 * log2(e)
  const float x2 = x * x;
  *x2out = x2;
  const float u = k0 * fmaf(k1 * x2, x, x);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(u * m2log2e));
}

ORION_DEVICE float gelu_tanh_f(float x) {
  float x2;
  return x * sigmoid2u_(x, &x2);
}

ORION_DEVICE float gelu_tanh_grad_f(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float x2;
  const float s = sigmoid2u_(x, &x2);
  // d/dx [x s(2u)] = s + x * 2 s (1 - s) * u'(x),  u' = k0 (1 + 3 k1 x^2)
  return fmaf(x * 2.f * s * (1.f - s), k0 * fmaf(3.f * k1, x2, 1.f), s);
}

ORION_DEVICE float silu_f(float x) { return x / (1.f + __expf(-x)); }

}  // namespace orion

#define HIP_LAUNCH_CHECK() (void)hipGetLastError()
