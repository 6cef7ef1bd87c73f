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

// [rows][32] bf16 image (64-byte rows, four 16-byte chunks): chunk c of row r at
// c ^ ((r >> 2) & 3).  ds_read_b128 of 32 consecutive rows at one chunk is conflict-free:
// each 16-lane group of the instruction covers 16 distinct (r & 3, slot) pairs.
ORION_DEVICE int loff32(int row, int col) {
  return row * 32 + ((((col >> 3) ^ (row >> 2)) & 3) << 3) + (col & 7);
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

// ---------------------------------------------------------------- LDS-DMA and asm LDS reads
// 16 bytes per lane global -> LDS (global_load_lds_dwordx4): the LDS destination is the
// wave-uniform base `l` + 16 * lane; the per-lane SOURCE address carries any swizzle.
ORION_DEVICE void glds16(const bf16_t* g, bf16_t* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

ORION_DEVICE unsigned lds_addr(const bf16_t* lds, int elem) {
  return (unsigned)(uintptr_t)((const __attribute__((address_space(3))) bf16_t*)(lds + elem));
}

// LDS reads as inline asm: reads the compiler cannot see, so its waitcnt pass does not
// drain an in-flight LDS-DMA ring (vmcnt(0)) before them, as it does before the builtin
// forms.  Completion is waited for by hand (s_waitcnt lgkmcnt(N)).
ORION_DEVICE bf16x4 tr_read(const bf16_t* lds, int elem) {
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(lds_addr(lds, elem)));
  return r;
}

// the same reads at a byte address + an immediate offset (loop-invariant per-lane bases)
template <int OFF>
ORION_DEVICE bf16x4 tr_read_at(unsigned a) {
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
  return r;
}
template <int OFF>
ORION_DEVICE bf16x8 b128_read_at(unsigned a) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
  return r;
}

ORION_DEVICE bf16x8 b128_read(const bf16_t* lds, int elem) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(lds_addr(lds, elem)));
  return r;
}

// tr_frag (above) on the asm read, [rows][D] image: element j of the lane's fragment is
// image row rbase + (i>>2) + rstep*(j>>2) + ... (see tr_frag)
template <int D = 128>
ORION_DEVICE bf16x8 tr_frag_asm(const bf16_t* img, int rbase, int cbase, int lane, int rstep = 8) {
  const int g = lane >> 4, i = lane & 15;
  const int row = rbase + (i >> 2);
  const int col = cbase + 16 * (g & 1) + 4 * (i & 3);
  return cat8(tr_read(img, loff<D>(row, col)), tr_read(img, loff<D>(row + rstep, col)));
}

// tr_frag_asm on an unswizzled [rows][32] image (64-byte rows: the 4 rows x 64 bytes a
// 32-lane half reads are one 256-byte bank row, conflict-free without a swizzle)
ORION_DEVICE bf16x8 tr_frag_asm_lin32(const bf16_t* img, int rbase, int lane, int rstep) {
  const int g = lane >> 4, i = lane & 15;
  const int row = rbase + (i >> 2);
  const int col = 16 * (g & 1) + 4 * (i & 3);
  return cat8(tr_read(img, row * 32 + col), tr_read(img, (row + rstep) * 32 + col));
}

// ---------------------------------------------------------------- buffer LDS-DMA
// A raw buffer resource over `bytes` bytes at `base` (gfx9 dword-3 format) and the 16-byte
// per-lane buffer_load_dwordx4 ... lds: LDS destination = wave-uniform `l` + 16 * lane;
// byte address = base + voff (per lane, carries any swizzle) + soff (wave-uniform).  The
// 32-bit per-lane offset costs one VGPR where global_load_lds needs a 64-bit pointer pair.
ORION_DEVICE __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

ORION_DEVICE void blds16(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff, bf16_t* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)l, 16, voff, soff,
                                           0, 0);
}

// wait until at most N LDS reads are outstanding; the fragments are "+v" operands so
// no MFMA reading them can be scheduled before the wait
template <int N, int TA>
ORION_DEVICE void lds_wait_frags(bf16x8 (&af)[TA], bf16x8 (&bf)[2]) {
  if constexpr (TA == 4) {
    asm volatile("s_waitcnt lgkmcnt(%6)"
                 : "+v"(af[0]), "+v"(af[1]), "+v"(af[2]), "+v"(af[3]), "+v"(bf[0]), "+v"(bf[1])
                 : "n"(N));
  } else if constexpr (TA == 2) {
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(af[0]), "+v"(af[1]), "+v"(bf[0]), "+v"(bf[1]) : "n"(N));
  } else {
    static_assert(TA == 1, "TA in {1, 2, 4}");
    asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(af[0]), "+v"(bf[0]), "+v"(bf[1]) : "n"(N));
  }
}

// Wave priority 1 while a wave issues an MFMA block (attention kernels): with 2-3 waves per
// SIMD the arbiter then feeds the matrix pipe first and the other waves' softmax / staging VALU
// fills the gaps.  Measured: Llama-shape backward -1.5 %, forward -1.3 %, GPT-2 step faster in
// 3 of 3 alternating pairs (profiles/ab/attn_setprio_r04.log).
#ifndef ORION_MFMA_PRIO
#define ORION_MFMA_PRIO 1  // wave priority while issuing MFMA blocks (0: off, A/B builds)
#endif
ORION_DEVICE void mfma_prio(bool on) {
  if constexpr (ORION_MFMA_PRIO > 0) {
    if (on) __builtin_amdgcn_s_setprio(ORION_MFMA_PRIO);
    else __builtin_amdgcn_s_setprio(0);
  }
}

template <int N>
ORION_DEVICE void wait_vm_exact() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

}  // namespace orion
