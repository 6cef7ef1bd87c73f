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

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_v;

// two floats -> one word of two bf16 (RNE) in ONE v_cvt_pk_bf16_f32; the OR of two scalar
// casts compiled to a cvt per value plus an and / shift / v_or_b32_sdwa repack
ORION_DEVICE unsigned pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2{lo, hi}), bf16x2_v));
}
ORION_DEVICE unsigned pack2_bf16(f32x2 v) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_v));
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
// 0.5 (1 + tanh(u)) == sigmoid(2u) = 1 / (1 + 2^z): one v_exp_f32 + one v_rcp_f32 instead of
// a tanhf expansion, with u = k0 (x + k1 x^3) and every constant folded into
// z = x (GELU_A + GELU_B x^2): GELU_A = -2 log2(e) k0, GELU_B = GELU_A k1 (k0 = sqrt(2/pi),
// k1 = 0.044715).  d/dx [x s] = s + s (1 - s) x (GELU_C + GELU_D x^2), GELU_C = 2 k0,
// GELU_D = 6 k0 k1.
constexpr float GELU_A = -2.302208198144325f, GELU_B = -0.1029432395800235f;
constexpr float GELU_C = 1.5957691216057308f, GELU_D = 0.21406444881780076f;

ORION_DEVICE float gelu_tanh_f(float x) {
  const float z = x * fmaf(x * x, GELU_B, GELU_A);
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z));
}

ORION_DEVICE float gelu_tanh_grad_f(float x) {
  const float x2 = x * x;
  const float s = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * fmaf(x2, GELU_B, GELU_A)));
  return fmaf(fmaf(-s, s, s), x * fmaf(x2, GELU_D, GELU_C), s);
}

// Two values per instruction (v_pk_mul / v_pk_fma / v_pk_add_f32) for the GEMM epilogues,
// where no MFMA runs beside the VALU (beside MFMAs packed f32 ops cost more than two single
// ones: MI355X_MICROARCH.md); the exp2 / rcp stay one per value.
ORION_DEVICE f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
ORION_DEVICE f32x2 splat2(float v) { return f32x2{v, v}; }
ORION_DEVICE f32x2 sigmoid2u_x2(f32x2 x, f32x2 x2) {
  const f32x2 z = x * fma2(x2, splat2(GELU_B), splat2(GELU_A));
  const f32x2 d = f32x2{__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)} + splat2(1.f);
  return f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
ORION_DEVICE f32x2 gelu_x2(f32x2 x) { return x * sigmoid2u_x2(x, x * x); }
// gelu(x) and GELU'(x) on one sigmoid
ORION_DEVICE void gelu_and_grad_x2(f32x2 x, f32x2& g, f32x2& d) {
  const f32x2 x2 = x * x, s = sigmoid2u_x2(x, x2);
  g = x * s;
  d = fma2(fma2(-s, s, s), x * fma2(x2, splat2(GELU_D), splat2(GELU_C)), s);
}
ORION_DEVICE f32x2 gelu_grad_x2(f32x2 x) {
  const f32x2 x2 = x * x, s = sigmoid2u_x2(x, x2);
  return fma2(fma2(-s, s, s), x * fma2(x2, splat2(GELU_D), splat2(GELU_C)), s);
}

ORION_DEVICE float silu_f(float x) { return x / (1.f + __expf(-x)); }

// sigmoid of a pair: 1 / (1 + 2^(-x log2 e)), one v_exp_f32 + one v_rcp_f32 per value
ORION_DEVICE f32x2 sigmoid2(f32x2 x) {
  const f32x2 z = x * splat2(-1.4426950408889634f);
  const f32x2 d = f32x2{__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)} + splat2(1.f);
  return f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

}  // namespace orion

#define HIP_LAUNCH_CHECK() (void)hipGetLastError()
