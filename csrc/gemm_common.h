// Shared pieces of the linear-layer GEMM kernels (csrc/gemm16.hip, csrc/wgrad.hip): argument
// block, epilogue kinds, the inline-asm LDS reads and barrier of the 16x16x32 kernels.
#pragma once

#include "mfma_lds.h"

namespace orion {

enum GemmEpi { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_GELU_BWD = 3, EPI_WGRAD = 4,
               EPI_SWIGLU_BWD = 5, EPI_EXP = 6, EPI_ROWSCALE = 7, EPI_ROPE = 8,
               EPI_SWIGLU = 9 };
constexpr int GEMM_DERIV = 0x100;  // orion_gemm's epi flag: GemmArgs::deriv

struct GemmArgs {
  const bf16_t* X;  long ldx;   // [M][K] row-major
  const bf16_t* W;  long ldw;   // NT: [N][K]; NN: [K][N]
  bf16_t* out;      long ldo;   // [M][N]
  const bf16_t* bias;           // [N]                      (EPI_BIAS, EPI_BIAS_GELU)
  bf16_t* out2;     long ldo2;  // gelu(a), [M][N]          (EPI_BIAS_GELU)
  const bf16_t* pre; long ldp;  // pre-activation a, [M][N] (EPI_GELU_BWD); the packed [M][2N]
                                // gate | up projection (EPI_SWIGLU_BWD: out = dgate, out2 = dup)
  int M, N, K, tiles_n;
  int flags;  // diagnostics (ORION_GEMM_DIAG, csrc/gemm.hip): 4 = stamped instantiation,
              // 32 = + stores waited for, 64 = one workgroup per work item (no persistent walk),
              // bits 8-15: m-tile group size of the work order (0 = 4)
  // split-K (EPI_WGRAD): work item = (k chunk of kchunk rows, tile)
  int kchunk, ksplit;
  float* slabs;          // ksplit > 1: fp32 partial tiles [ksplit][M][N]
  const float* scale;    // ksplit == 1: out (fp32 when out_f32, else bf16) = acc * *scale
  int accumulate, out_f32;  //            (+ the value already in out when accumulate)
  // EPI_GELU_BWD: fp32 column sums of the result (the bias gradient)
  // per 64-row block, colsum[ceil(M / 64)][N]; null = none
  float* colsum;
  // LM head + cross-entropy (csrc/lmhead.hip).  EPI_EXP (forward, NT): out = exp(acc - *cref)
  // (bf16), rowpart[m][n / 128] = fp32 sum of those over the wave's 128 columns, tlog[m] =
  // acc at column tgt[m].  EPI_ROWSCALE (input gradient): out = rs[m] acc (the softmax's
  // 1 / Z per row; the one-hot term is folded into the exp tile by the fold kernel).
  float* rowpart; int npart;
  const int64_t* tgt;
  float* tlog;
  const float* cref;
  const float* rs;
  // GELU derivative stored instead of the pre-activation (GPT-2 MLP, round 5): EPI_BIAS_GELU
  // writes GELU'(a) as its first output, EPI_GELU_BWD multiplies by pre as given
  int deriv;
  // EPI_ROPE (Llama's packed QKV projection, round 6): columns [0, rcols) are heads of rD = 128
  // rotated by RoPE in the rotate-half form -- pair (d, d + rD / 2) of row m at position
  // (m % rT) + rpos0 with the fp32 tables rcos / rsin [pos][rD / 2] -- before the bf16 store
  const float* rcos;
  const float* rsin;
  int rT, rpos0, rcols, rD;
  // EPI_SWIGLU (Llama's gate_up projection, round 6): N = 2F, W = [W_gate; W_up] [2F][K].  The
  // wave owning tile columns [nw, nw + 128) computes gate features f = nw / 2 + [0, 64) in its
  // first 64 columns and the matching up rows F + f in the last 64 (the W stream reads those
  // rows), so silu(gate) * up is lane-local: out = the packed gate | up projection [M][2F] in
  // its natural layout, out2 = h [M][F]
};

// ---- 16x16x32 kernel helpers (csrc/gemm16.hip)
// LDS reads as inline asm (the compiler's wait-count pass cannot see them, so an in-flight
// LDS-DMA ring is not drained before each read); completion is waited for by hand.
ORION_DEVICE int nt_swz(int r) { return (r >> 1) & 7; }
ORION_DEVICE int km_swz(int k) { return ((k >> 1) & 1) | (((k >> 3) & 1) << 1); }

template <int OFF>
ORION_DEVICE bf16x8 rd_b128(unsigned a) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
  return r;
}

template <int OFF>
ORION_DEVICE bf16x4 rd_tr(unsigned a) {
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(OFF));
  return r;
}

ORION_DEVICE f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, a),
                                                 __builtin_bit_cast(bf16x8_mfma, b), c, 0, 0, 0);
}

ORION_DEVICE void g_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// all fragment reads of the phase retired; the fragments become "+v" operands of the wait so
// no MFMA that uses them is scheduled above it
ORION_DEVICE void g_wait_lds(bf16x8 (&a)[4][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0][0]), "+v"(a[0][1]), "+v"(a[1][0]), "+v"(a[1][1]), "+v"(a[2][0]),
                 "+v"(a[2][1]), "+v"(a[3][0]), "+v"(a[3][1]));
}

// csrc/gemm16.hip: forward / input gradient (gemm16) and weight gradient (gemm16_wgrad);
// gemm16_ok: the work item's 32-bit buffer offsets (one 256-row band, the whole k-major W)
bool gemm16_ok(const GemmArgs& a, int wkm);
int gemm16(const GemmArgs& a, int wkm, int epi, hipStream_t st);
int gemm16_wgrad(const GemmArgs& a, int bt, hipStream_t st);

}  // namespace orion
