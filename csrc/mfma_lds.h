// MFMA operand / LDS-image helpers shared by the attention and GEMM kernels (gfx950).
//
// v_mfma_f32_32x32x16_bf16: A 32x16, B 16x32, C 32x32 with
// C[row = (r&3) + 8(r>>2) + 4(lane>>5)][col = lane&31].
//
// LDS images: 16-byte chunk c of row r of a [rows][D] bf16 tile lives at chunk
// c ^ swz<D>(r); the XOR makes both row reads (ds_read_b128) and transposed reads
// (ds_read_b64_tr_b16, 4 rows x 16 columns per 16-lane group) conflict-free.
#pragma once

#include "common.h"

namespace orion {

template <int D>
ORION_DEVICE int swz(int r) {
  if constexpr (D == 128) {
    return ((r & 3) << 2) | ((r >> 2) & 3);
  } else {
    return (((r >> 1) & 1) << 2) | (((r >> 3) & 1) << 1) | ((r >> 2) & 1);
  }
}

// element offset of (row, col) in a swizzled [rows][D] bf16 image
template <int D>
ORION_DEVICE int loff(int row, int col) {
  return row * D + ((((col >> 3) ^ swz<D>(row))) << 3) + (col & 7);
}

ORION_DEVICE bf16x8 lds_b128(const bf16_t* base, int off) {
  return *reinterpret_cast<const bf16x8*>(base + off);
}

typedef __attribute__((ext_vector_type(4))) short s16x4;

ORION_DEVICE bf16x4 lds_tr(const bf16_t* base, int off) {
  typedef __attribute__((address_space(3))) s16x4 lds_s4;
  s16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + off));
  return __builtin_bit_cast(bf16x4, r);
}

ORION_DEVICE bf16x8 cat8(bf16x4 lo, bf16x4 hi) {
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

ORION_DEVICE f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_mfma, a),
                                                 __builtin_bit_cast(bf16x8_mfma, b), c, 0, 0, 0);
}

ORION_DEVICE f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// 16 fp32 accumulator registers rr = 8s..8s+7 -> one bf16 MFMA fragment
ORION_DEVICE bf16x8 acc_to_frag(const f32x16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(x[8 * s + j]);
  return r;
}

// Transposed 8-element fragment of a swizzled [rows][D] image:
// element j of lane (group g = lane>>4, i = lane&15) is image[row0 + 8*(j>>2) + (j&3)][col]
// with row0 = rbase + (i>>2) supplied per lane and col = cbase + 16*(g&1) + 4*(i&3).
template <int D>
ORION_DEVICE bf16x8 tr_frag(const bf16_t* img, int rbase, int cbase, int lane, int rstep) {
  const int g = lane >> 4, i = lane & 15;
  const int row = rbase + (i >> 2);
  const int col = cbase + 16 * (g & 1) + 4 * (i & 3);
  return cat8(lds_tr(img, loff<D>(row, col)), lds_tr(img, loff<D>(row + rstep, col)));
}

}  // namespace orion
