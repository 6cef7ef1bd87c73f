// Weight-gradient GEMM for gfx950: dW[n1][n2] = sum_m dY[m][n1] * X[m][n2].
//
// The reduction runs over all tokens (m = 65,536 for the GPT-2 bench) into a small
// output (768..3072 x 768), with BOTH operands stored k-major ([m][n] row-major).
// hipBLASLt's solutions for this "TN, tiny output, huge K" regime measure
// 0.64-0.96 PF/s on MI355X (scripts/bench_gemms.py).  This kernel is built for it:
//
//   * 256 x 256 output tile per 8-wave workgroup (waves 2 (n1) x 4 (n2), 128 x 64
//     each = 4 x 2 v_mfma_f32_32x32x16_bf16 accumulators): each 32-row stage
//     (32 KB of operands) feeds 128 MFMAs, 128 FLOP per byte of L2 traffic;
//   * both operands reach the MFMA through ds_read_b64_tr_b16 (the gfx950
//     transposing LDS read) from XOR-swizzled [32][128] images, i.e. the k-major
//     global layout is consumed as is -- no transpose pass, and the same k
//     permutation on A and B keeps the product exact;
//   * split-K over token chunks sized so the grid is ~one workgroup per CU (128 KB
//     LDS ring), partial tiles go to fp32 slabs folded by
//     slab_sum (activations.hip), or straight to bf16 when no split is needed;
//   * XCD-aware block -> (k-chunk, tile) mapping: the workgroups of one k-chunk sit
//     on one XCD, so its 4 MB L2 serves the shared operand rows to all of them;
//   * LDS-DMA staging into a 4-deep ring (see the kernel comment), one raw barrier
//     per stage.
#include "mfma_lds.h"

namespace orion {

constexpr int WG_T = 512;          // 8 waves: 2 along n1 x 4 along n2
constexpr int WG_BK = 32;          // m rows per stage
constexpr int WG_NS = 4;           // LDS ring depth (3 stages in flight during compute)
constexpr int IMG = WG_BK * 128;   // one [32][128] bf16 image (8 KB)
constexpr int WG_STAGE = 4 * IMG;  // A halves 0,1 | B halves 0,1 = 32 KB

ORION_DEVICE void glds16(const bf16_t* g, bf16_t* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// ds_read_b64_tr_b16 as inline asm: LDS reads the compiler cannot see, so its waitcnt
// pass does not drain the in-flight LDS-DMA ring (vmcnt(0)) before them (the builtin
// form gets exactly that).  Completion is waited for by hand: lds_wait() below.
ORION_DEVICE bf16x4 tr_read(const bf16_t* lds, int elem) {
  const unsigned addr =
      (unsigned)(uintptr_t)((const __attribute__((address_space(3))) bf16_t*)(lds + elem));
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}

// tr_frag (mfma_lds.h) on the asm read
ORION_DEVICE bf16x8 tr_frag_asm(const bf16_t* img, int rbase, int cbase, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int row = rbase + (i >> 2);
  const int col = cbase + 16 * (g & 1) + 4 * (i & 3);
  return cat8(tr_read(img, loff<128>(row, col)), tr_read(img, loff<128>(row + 8, col)));
}

ORION_DEVICE void wait_vm(int n) {  // retire all but the newest n vector-memory ops of this wave
  if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Staging is LDS-DMA (global_load_lds_dwordx4): no VGPRs, so a 4-deep ring keeps
// ~96 KB per CU in flight -- the register-staged versions (32-48 KB in flight)
// ran latency-bound at ~0.8 PF/s.  A wave-instruction writes 1 KB lane-linearly
// (4 rows of one 128-column image); the XOR swizzle of the image is applied to the
// per-lane SOURCE column instead.  Barriers are raw s_barrier with counted vmcnt
// (a __syncthreads() would drain every in-flight stage).
__global__ __launch_bounds__(WG_T) void wgrad_kernel(
    const bf16_t* __restrict__ A, long lda, const bf16_t* __restrict__ B, long ldb, int M, int N1,
    int N2, int tiles_n2, int ntiles, int chunk, float* __restrict__ slabs,
    bf16_t* __restrict__ out, const float* __restrict__ scale) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];  // [WG_NS stages][A0 A1 B0 B1]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h32 = lane >> 5;
  const int wr = wv >> 2, wc = wv & 3;

  // bijective XCD remap (blocks bid, bid+8, ... share an XCD)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int kc = wid / ntiles, tile = wid % ntiles;
  const int n10 = (tile / tiles_n2) * 256, n20 = (tile % tiles_n2) * 256;
  const int m0 = kc * chunk;
  const int nsteps = (min(M, m0 + chunk) - m0) / WG_BK;

  // this wave's two 1-KB blocks of each operand per stage: block blk covers image half
  // blk>>3, rows 4*(blk&7)..+3; lane -> row +lane/16, LDS slot lane%16 = source chunk ^ swz
  long goffA[2], goffB[2];
  int loffs[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = wv * 2 + i, half = blk >> 3;
    const int row = 4 * (blk & 7) + (lane >> 4), slot = lane & 15;
    const int col = half * 128 + 8 * (slot ^ swz<128>(row));
    goffA[i] = (long)row * lda + min(n10 + col, N1 - 8);
    goffB[i] = (long)row * ldb + min(n20 + col, N2 - 8);
    loffs[i] = half * IMG + (blk & 7) * 512;
  }
  auto issue = [&](int step) {
    bf16_t* base = smem + (step % WG_NS) * WG_STAGE;
    const long mr = m0 + (long)step * WG_BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      glds16(A + mr * lda + goffA[i], base + loffs[i]);
      glds16(B + mr * ldb + goffB[i], base + 2 * IMG + loffs[i]);
    }
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = zero16();

  const int pre = min(nsteps, WG_NS - 1);
  for (int st = 0; st < pre; ++st) issue(st);
  for (int t = 0; t < nsteps; ++t) {
    wait_vm(4 * min(nsteps - 1 - t, WG_NS - 2));  // this wave's share of stage t has landed
    asm volatile("s_barrier" ::: "memory");        // ... and every other wave's; stage t-1 is free
    if (t + WG_NS - 1 < nsteps) issue(t + WG_NS - 1);  // refill the slot stage t-1 used
    const bf16_t* As = smem + (t % WG_NS) * WG_STAGE + wr * IMG;
    const bf16_t* Bs = smem + (t % WG_NS) * WG_STAGE + 2 * IMG + (wc >> 1) * IMG;
    // both k16 steps' fragments are requested up front (24 reads); the first step's
    // MFMAs start once its 12 reads have returned (lgkmcnt counts in issue order)
    bf16x8 af[2][4], bfr[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int a = 0; a < 4; ++a) af[s][a] = tr_frag_asm(As, 16 * s + 4 * h32, a * 32, lane);
#pragma unroll
      for (int b = 0; b < 2; ++b) bfr[s][b] = tr_frag_asm(Bs, 16 * s + 4 * h32, (wc & 1) * 64 + b * 32, lane);
    }
    // the "+v" operands pin every MFMA that reads a fragment after its wait
    asm volatile("s_waitcnt lgkmcnt(12)"
                 : "+v"(af[0][0]), "+v"(af[0][1]), "+v"(af[0][2]), "+v"(af[0][3]), "+v"(bfr[0][0]),
                   "+v"(bfr[0][1]));
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[a][b] = mfma32(af[0][a], bfr[0][b], acc[a][b]);
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(af[1][0]), "+v"(af[1][1]), "+v"(af[1][2]), "+v"(af[1][3]), "+v"(bfr[1][0]),
                   "+v"(bfr[1][1]));
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[a][b] = mfma32(af[1][a], bfr[1][b], acc[a][b]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue: C[row = (r&3)+8(r>>2)+4*h32][col = lane&31] of each 32x32 accumulator
  const int l32 = lane & 31;
  const float sc = (!slabs && scale) ? *scale : 1.f;
  float* sl = slabs ? slabs + (long)kc * N1 * N2 : nullptr;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n2 = n20 + wc * 64 + b * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n1 = n10 + wr * 128 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32;
        if (n1 < N1 && n2 < N2) {
          if (sl) sl[(long)n1 * N2 + n2] = acc[a][b][r];
          else out[(long)n1 * N2 + n2] = f2bf(acc[a][b][r] * sc);
        }
      }
    }
}

}  // namespace orion

using namespace orion;

// Split count: minimise (rounds of one-workgroup-per-CU) x (rows per workgroup) plus
// the fp32 slab round trip, in units of rows of work.
int orion_wgrad_splits(int M, int N1, int N2) {
  const long tiles = (long)((N1 + 255) / 256) * ((N2 + 255) / 256);
  const double ns_per_row = 22.0;  // one 256x256x1 slice at ~60 % of the MFMA rate
  double best = 1e30;
  int bestS = 1;
  for (int S = 1; S <= 32; ++S) {
    const int chunk = ((M / WG_BK + S - 1) / S) * WG_BK;
    if (chunk < 8 * WG_BK && S > 1) break;
    const int Se = (M + chunk - 1) / chunk;
    if (Se != S) continue;
    const long rounds = (tiles * Se + 255) / 256;  // one workgroup per CU (128 KB LDS)
    double cost = (double)rounds * chunk;
    if (Se > 1) cost += (double)Se * N1 * N2 * 8.0 / 5e12 * 1e9 / ns_per_row;
    if (cost < best * 0.98) {
      best = cost;
      bestS = Se;
    }
  }
  return bestS;
}

// number of k-chunks actually produced when S are requested (chunks are whole stages)
int orion_wgrad_effective_splits(int M, int S) {
  if (S < 1) S = 1;
  const int chunk = ((M / WG_BK + S - 1) / S) * WG_BK;
  return chunk > 0 ? (M + chunk - 1) / chunk : 1;
}

int orion_wgrad_lds() { return WG_NS * WG_STAGE * (int)sizeof(bf16_t); }

// A (M x N1, ld lda), B (M x N2, ld ldb) bf16 -> slabs (S, N1, N2) fp32 when S > 1
// (caller folds them), else out (N1, N2) bf16 scaled by *scale (nullable).
int orion_wgrad(const void* A, long lda, const void* B, long ldb, int M, int N1, int N2, int S,
                float* slabs, void* out, const float* scale, hipStream_t st) {
  if (M % WG_BK || N1 % 8 || N2 % 8 || lda % 8 || ldb % 8 || N1 < 8 || N2 < 8) return -1;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -2;
  const int chunk = ((M / WG_BK + S - 1) / S) * WG_BK;
  const int Se = (M + chunk - 1) / chunk;
  if (Se != S) return -3;
  if (S > 1 && !slabs) return -4;
  const int t1 = (N1 + 255) / 256, t2 = (N2 + 255) / 256;
  const int ntiles = t1 * t2;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)wgrad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            orion_wgrad_lds()) != hipSuccess)
      return -5;
    attr = true;
  }
  wgrad_kernel<<<ntiles * S, WG_T, orion_wgrad_lds(), st>>>(
      (const bf16_t*)A, lda, (const bf16_t*)B, ldb, M, N1, N2, t2, ntiles, chunk,
      S > 1 ? slabs : nullptr, (bf16_t*)out, scale);
  return (int)hipGetLastError();
}
