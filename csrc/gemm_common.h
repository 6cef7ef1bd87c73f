// Shared pieces of the linear-layer GEMM kernels (csrc/gemm.hip, csrc/gemm_phased.hip):
// argument block, epilogue kinds and the C^T-tile epilogue (bias / GELU / GELU-backward,
// 16-byte row stores after one v_permlane32_swap per register pair).
#pragma once

#include "mfma_lds.h"

namespace orion {

enum GemmEpi { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_GELU_BWD = 3, EPI_WGRAD = 4 };

struct GemmArgs {
  const bf16_t* X;  long ldx;   // [M][K] row-major
  const bf16_t* W;  long ldw;   // NT: [N][K]; NN: [K][N]
  bf16_t* out;      long ldo;   // [M][N]
  const bf16_t* bias;           // [N]                      (EPI_BIAS, EPI_BIAS_GELU)
  bf16_t* out2;     long ldo2;  // gelu(a), [M][N]          (EPI_BIAS_GELU)
  const bf16_t* pre; long ldp;  // pre-activation a, [M][N] (EPI_GELU_BWD)
  int M, N, K, tiles_n;
  int flags;  // diagnostics (ORION_GEMM_DIAG): 1 = no LDS-DMA after the first stage; 2 = DMA spread over
              // k steps (csrc/gemm.hip only); 8 = no C stores;
              // 16 = gemm_phased.hip's 4-quadrant schedule (ORION_GEMM_CFG / ORION_WGRAD_CFG = 8)
  // split-K (EPI_WGRAD, csrc/gemm_phased.hip): work item = (k chunk of kchunk rows, tile)
  int kchunk, ksplit;
  float* slabs;          // ksplit > 1: fp32 partial tiles [ksplit][M][N]
  const float* scale;    // ksplit == 1: out (fp32 when out_f32, else bf16) = acc * *scale
  int accumulate, out_f32;  //            (+ the value already in out when accumulate)
  // EPI_GELU_BWD (csrc/gemm_phased.hip): fp32 column sums of the result (the bias gradient)
  // per 64-row block, colsum[ceil(M / 64)][N]; null = none
  float* colsum;
};

// Epilogue math of one 32 x 32 accumulator of C^T (rows n = nb + (r&3) + 8(r>>2) + 4 h32,
// column = the lane's output row m, clamped to mc): fp32 bias / GELU / GELU-backward, one bf16
// rounding, packed pairs pk[g4][0..1] = columns nb + 8 g4 + 4 h32 + 0..3.  GELU2 = 1: the
// second output of EPI_BIAS_GELU (gelu(a)) instead of the first (a).  EPI_GELU_BWD multiplies by
// GELU'(pre + bias) (bias optional).  vals (if given): the 16 fp32 values before rounding.
template <int EPI, bool GELU2 = false>
ORION_DEVICE void gemm_epi_values(const GemmArgs& g, const f32x16& acc, int mc, int nb, int h32,
                                  unsigned (&pk)[4][2], float* vals = nullptr) {
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int n = nb + 8 * g4 + 4 * h32;
    const int nc = n < g.N ? n : 0;  // N % 8 == 0: a 4-run is all in or all out
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = acc[4 * g4 + e];
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
      const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(g.bias + nc);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += bf2f(b4[e]);
    }
    if constexpr (EPI == EPI_GELU_BWD) {
      ORION_DASSERT(mc < g.M && nc + 4 <= g.N);
      const bf16x4 a4 = *reinterpret_cast<const bf16x4*>(g.pre + (long)mc * g.ldp + nc);
      float pb[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) pb[e] = bf2f(a4[e]);
      if (g.bias) {
        const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(g.bias + nc);
#pragma unroll
        for (int e = 0; e < 4; ++e) pb[e] += bf2f(b4[e]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] *= gelu_tanh_grad_f(pb[e]);
    }
    if constexpr (GELU2) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = gelu_tanh_f(v[e]);
    }
    if (vals) {
#pragma unroll
      for (int e = 0; e < 4; ++e) vals[4 * g4 + e] = v[e];
    }
    pk[g4][0] = pack_bf16x2(v[0], v[1]);
    pk[g4][1] = pack_bf16x2(v[2], v[3]);
  }
}

// register pairs (2 pr, 2 pr + 1) after one v_permlane32_swap each: lanes 0-31 hold columns
// 16 pr .. 16 pr + 7 and lanes 32-63 columns 16 pr + 8 .. 16 pr + 15 of the lane's row
ORION_DEVICE uint4 gemm_epi_swap(const unsigned (&pp)[4][2], int pr) {
  const auto r0 = __builtin_amdgcn_permlane32_swap(pp[2 * pr][0], pp[2 * pr + 1][0], false, false);
  const auto r1 = __builtin_amdgcn_permlane32_swap(pp[2 * pr][1], pp[2 * pr + 1][1], false, false);
  uint4 w;
  w.x = r0[0]; w.y = r1[0]; w.z = r0[1]; w.w = r1[1];
  return w;
}

// One 32 x 32 accumulator of C^T through the epilogue and out as 16-byte row segments
// (gemm.hip's kernels: 32 rows x 32 bytes per store instruction).
template <int EPI>
ORION_DEVICE void gemm_epilogue_tile(const GemmArgs& g, const f32x16& acc, int m, int mc, int nb,
                                     int h32) {
  auto store = [&](const unsigned (&pp)[4][2], bf16_t* base, long ld) {
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      const uint4 w = gemm_epi_swap(pp, pr);
      const int n = nb + 16 * pr + 8 * h32;
      if (m < g.M && n < g.N && !(g.flags & 8)) {  // flags & 8: diagnostic, no C stores
        ORION_DASSERT(n + 8 <= g.N && m >= 0);
        *reinterpret_cast<uint4*>(base + (long)m * ld + n) = w;
      }
    }
  };
  unsigned pk[4][2];
  gemm_epi_values<EPI>(g, acc, mc, nb, h32, pk);
  store(pk, g.out, g.ldo);
  if constexpr (EPI == EPI_BIAS_GELU) {
    gemm_epi_values<EPI, true>(g, acc, mc, nb, h32, pk);
    store(pk, g.out2, g.ldo2);
  }
}

// The whole 256 x 256 C tile of a workgroup (8 waves: grp = n half, wm = 64-row m block,
// acc[i][j] = C^T tile of n 32 i, m 32 j) staged through LDS so that every store instruction
// writes two whole 512-byte row segments (eight full 128-byte lines) instead of 32 rows x 32
// bytes.  LDS image [256 m][256 n] bf16, 16-byte chunk c of row r at c ^ (r & 15): the b128
// writes (16 rows at one chunk) and the row reads (consecutive chunks) are conflict-free.
// Needs 128 KB of LDS no longer read by anyone (caller's barrier) and no LDS-DMA in flight.
template <int EPI>
ORION_DEVICE void gemm_epilogue_lds(const GemmArgs& g, const f32x16 (&acc)[4][2], bf16_t* smem, int m0,
                                    int n0, int wm, int grp, int wv, int lane) {
  const int h32 = lane >> 5, l32 = lane & 31;
  char* lds = reinterpret_cast<char*>(smem);
  auto fill = [&](auto gelu2) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = wm * 64 + j * 32 + l32;
      const int mc = min(m0 + r, g.M - 1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        unsigned pk[4][2];
        gemm_epi_values<EPI, decltype(gelu2)::value>(g, acc[i][j], mc, n0 + grp * 128 + i * 32, h32, pk);
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          const int c = grp * 16 + i * 4 + 2 * pr + h32;
          *reinterpret_cast<uint4*>(lds + (r * 32 + (c ^ (r & 15))) * 16) = gemm_epi_swap(pk, pr);
        }
      }
    }
  };
  auto drain = [&](bf16_t* base, long ld) {
#pragma unroll 4
    for (int it = 0; it < 16; ++it) {
      const int r = 2 * (wv + 8 * it) + h32, c = l32;
      const uint4 w = *reinterpret_cast<const uint4*>(lds + (r * 32 + (c ^ (r & 15))) * 16);
      const int m = m0 + r, n = n0 + 8 * c;
      if (m < g.M && n < g.N && !(g.flags & 8)) {
        ORION_DASSERT(n + 8 <= g.N);
        *reinterpret_cast<uint4*>(base + (long)m * ld + n) = w;
      }
    }
  };
  fill(std::false_type());
  __syncthreads();
  drain(g.out, g.ldo);
  if constexpr (EPI == EPI_BIAS_GELU) {
    __syncthreads();
    fill(std::true_type());
    __syncthreads();
    drain(g.out2, g.ldo2);
  }
}

// csrc/gemm_phased.hip
bool gemm_phased_ok(const GemmArgs& a, int wkm);
int gemm_phased(const GemmArgs& a, int wkm, int epi, hipStream_t st);
// weight gradient out[M][N] = sum_k X[k][M] W[k][N] (both operands k-major), split-K
int gemm_phased_wgrad(const GemmArgs& a, hipStream_t st);
// csrc/gemm16.hip: the same operations on v_mfma_f32_16x16x32_bf16 (same requirements as
// gemm_phased_ok, plus 8-element aligned pre-activation rows for EPI_GELU_BWD)
bool gemm16_ok(const GemmArgs& a, int wkm);
int gemm16(const GemmArgs& a, int wkm, int epi, hipStream_t st);
int gemm16_wgrad(const GemmArgs& a, hipStream_t st);

}  // namespace orion
