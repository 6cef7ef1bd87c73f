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
#include "gemm_common.h"

namespace orion {


// Staging is LDS-DMA (global_load_lds_dwordx4): no VGPRs, so a ring of NS stages
// keeps NS-1 stages per CU in flight (register staging held 32-48 KB and ran
// latency-bound at ~0.8 PF/s).  A wave-instruction writes 1 KB lane-linearly (4
// rows of one 128-column image); the image's XOR swizzle is applied to the per-lane
// SOURCE column instead.  Barriers are raw s_barrier with counted vmcnt (a
// __syncthreads() would drain every in-flight stage).  Inside a stage the fragment
// reads of k16 step s+1 are issued before the MFMAs of step s (sched_barrier keeps
// the compiler from regrouping them).
// KS k16 steps (16 rows each) per stage, NS-deep ring, WM waves along n1 (each owning
// 256/WM rows = TA MFMA tiles) x 4 waves along n2 (64 columns each)
template <int KS, int NS, int WM>
__global__ __launch_bounds__(WM * 256) void wgrad_kernel(
    const bf16_t* __restrict__ A, long lda, const bf16_t* __restrict__ B, long ldb, int M, int N1,
    int N2, int tiles_n2, int ntiles, int chunk, float* __restrict__ slabs,
    void* __restrict__ out, const float* __restrict__ scale, int accumulate, int out_f32) {
  constexpr int BK = 16 * KS;        // m rows per stage
  constexpr int IMG = BK * 128;      // one [BK][128] image
  constexpr int STAGE = 4 * IMG;     // A halves 0,1 | B halves 0,1
  constexpr int NW = WM * 4;          // waves
  constexpr int TA = 8 / WM;          // 32-row MFMA tiles per wave along n1
  constexpr int BPW = KS * 8 / NW;    // 1-KB blocks per wave per operand per stage
  static_assert(BPW * NW == KS * 8, "stage blocks must divide over the waves");
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
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
  const int nsteps = (min(M, m0 + chunk) - m0) / BK;

  // block blk (0 .. 8*KS-1) of an operand: image half blk / (4*KS), rows 4*(blk % (4*KS))..+3;
  // lane -> row + lane/16, LDS slot lane%16 = source chunk ^ swz(row)
  long goffA[BPW], goffB[BPW];
  int loffs[BPW];
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    const int blk = wv * BPW + i, half = blk / (4 * KS), rb4 = blk % (4 * KS);
    const int row = 4 * rb4 + (lane >> 4), slot = lane & 15;
    const int col = half * 128 + 8 * (slot ^ swz<128>(row));
    goffA[i] = (long)row * lda + min(n10 + col, N1 - 8);
    goffB[i] = (long)row * ldb + min(n20 + col, N2 - 8);
    loffs[i] = half * IMG + rb4 * 512;
  }
  auto issue = [&](int step) {
    bf16_t* base = smem + (step % NS) * STAGE;
    const long mr = m0 + (long)step * BK;
#pragma unroll
    for (int i = 0; i < BPW; ++i) {
      ORION_DASSERT(mr + BK <= M && goffA[i] % lda + 8 <= N1 && goffB[i] % ldb + 8 <= N2);
      glds16(A + mr * lda + goffA[i], base + loffs[i]);
      glds16(B + mr * ldb + goffB[i], base + 2 * IMG + loffs[i]);
    }
  };

  f32x16 acc[TA][2];
#pragma unroll
  for (int a = 0; a < TA; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = zero16();

  const int pre = min(nsteps, NS - 1);
  for (int st = 0; st < pre; ++st) issue(st);
  for (int t = 0; t < nsteps; ++t) {
    // this wave's share of stage t has landed (stages t+1 .. t+NS-2 may stay in flight)
    const int ahead = min(nsteps - 1 - t, NS - 2);
    constexpr int PS = 2 * BPW;  // glds instructions per stage per wave
    if constexpr (NS >= 8) {
      if (ahead >= 6) wait_vm_exact<6 * PS>();
      else if (ahead == 5) wait_vm_exact<5 * PS>();
      else if (ahead == 4) wait_vm_exact<4 * PS>();
      else if (ahead == 3) wait_vm_exact<3 * PS>();
      else if (ahead == 2) wait_vm_exact<2 * PS>();
      else if (ahead == 1) wait_vm_exact<PS>();
      else wait_vm_exact<0>();
    } else if constexpr (NS >= 4) {
      if (ahead >= 2) wait_vm_exact<2 * PS>();
      else if (ahead == 1) wait_vm_exact<PS>();
      else wait_vm_exact<0>();
    } else if constexpr (NS == 3) {
      if (ahead >= 1) wait_vm_exact<PS>();
      else wait_vm_exact<0>();
    } else {
      wait_vm_exact<0>();
    }
    asm volatile("s_barrier" ::: "memory");  // every wave's share landed; slot of stage t-1 free
    if (t + NS - 1 < nsteps) issue(t + NS - 1);
    const bf16_t* As = smem + (t % NS) * STAGE + (wr * TA * 32 / 128) * IMG;
    const bf16_t* Bs = smem + (t % NS) * STAGE + 2 * IMG + (wc >> 1) * IMG;
    bf16x8 af[2][TA], bfr[2][2];
    auto fetch = [&](int s, int slot) {
#pragma unroll
      for (int a = 0; a < TA; ++a)
        af[slot][a] = tr_frag_asm(As, 16 * s + 4 * h32, (wr * TA * 32) % 128 + a * 32, lane);
#pragma unroll
      for (int b = 0; b < 2; ++b)
        bfr[slot][b] = tr_frag_asm(Bs, 16 * s + 4 * h32, (wc & 1) * 64 + b * 32, lane);
    };
    fetch(0, 0);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int cur = s & 1;
      if (s + 1 < KS) {
        fetch(s + 1, cur ^ 1);
        lds_wait_frags<2 * (TA + 2), TA>(af[cur], bfr[cur]);  // step s = the older half
      } else {
        lds_wait_frags<0, TA>(af[cur], bfr[cur]);
      }
#pragma unroll
      for (int a = 0; a < TA; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma32(af[cur][a], bfr[cur][b], acc[a][b]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // epilogue: C[row = (r&3)+8(r>>2)+4*h32][col = lane&31] of each 32x32 accumulator
  const int l32 = lane & 31;
  const float sc = (!slabs && scale) ? *scale : 1.f;
  float* sl = slabs ? slabs + (long)kc * N1 * N2 : nullptr;
#pragma unroll
  for (int a = 0; a < TA; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n2 = n20 + wc * 64 + b * 32 + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n1 = n10 + wr * TA * 32 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h32;
        if (n1 < N1 && n2 < N2) {
          ORION_DASSERT(n1 >= 0 && n2 >= 0);
          if (sl) sl[(long)n1 * N2 + n2] = acc[a][b][r];
          else {
            const long o = (long)n1 * N2 + n2;
            float v = acc[a][b][r] * sc;
            if (accumulate) v += load_grad(out, o, out_f32);  // accumulation into the arena
            store_grad(out, o, v, out_f32);
          }
        }
      }
    }
}

}  // namespace orion

using namespace orion;

// Two kernels serve the weight gradients:
//   * csrc/gemm16.hip (EPI_WGRAD work items: k chunk x tile, v_mfma_f32_16x16x32_bf16,
//     persistent walk) for every token count that is a multiple of 64 -- GPT-2 weight
//     gradients 4.9 vs 5.6 ms for the 32x32x16 kernels it replaced, whole step +3.9 %;
//   * wgrad_kernel above (32-row stages, configuration KS 2 / NS 4 / 16 waves) for the rest.
// Round 4 removed the other wgrad_kernel configurations and the 32x32x16 phased kernel (no
// default path selected them) and the per-call ORION_WGRAD_CFG lookup.
constexpr int WG_KS = 2, WG_NS = 4, WG_WM = 4;

static int wg_bk(int M) { return M % 64 ? 16 * WG_KS : 64; }

// Split count: minimise (rounds of one-workgroup-per-CU) x (rows per workgroup) plus
// the fp32 slab round trip, in units of rows of work.
int orion_wgrad_splits(int M, int N1, int N2) {
  const long tiles = (long)((N1 + 255) / 256) * ((N2 + 255) / 256);
  const double ns_per_row = 22.0;  // one 256x256x1 slice at ~60 % of the MFMA rate
  double best = 1e30;
  int bestS = 1;
  for (int S = 1; S <= 32; ++S) {
    const int BK = wg_bk(M);
    const int chunk = ((M / BK + S - 1) / S) * BK;
    if (chunk < 8 * BK && S > 1) break;
    const int Se = (M + chunk - 1) / chunk;
    if (Se != S) continue;
    const long rounds = (tiles * Se + 255) / 256;  // one workgroup per CU
    double cost = (double)rounds * chunk;
    if (Se > 1) cost += (double)Se * N1 * N2 * 8.0 / 5e12 * 1e9 / ns_per_row;
    if (cost < best * 0.98) {
      best = cost;
      bestS = Se;
    }
  }
  return bestS;
}

// Tail split of an unsplit weight gradient whose tile count leaves a partial last round
// (one workgroup per CU, 256 CUs): the first R1 output rows -- the whole rows of tiles that
// fit in the whole rounds -- run unsplit; the remaining rows (at most ~half a round of tiles,
// the last row of tiles may be partial) run split-K over S2 = 256 / tail-tiles chunks, so the
// last round costs about 1 / S2 of an item instead of a whole one.
// Llama-7B gate_up (22,016 x 4,096: 1,376 tiles, 5.4 rounds): 80 rows of tiles unsplit +
// 6 rows at S2 = 2 -- 5.5 instead of 6 item times.  GPT-2's LM head (50,304 x 768: 591
// tiles, 2.3 rounds, round 5): 170 rows unsplit (510 tiles) + 26.5 rows at S2 = 3 -- 2.33
// instead of 3 item times.  Returns R1 (0: no split) and S2.
int orion_wgrad_effective_splits(int M, int S);

int orion_wgrad_tail_rows(int M, int N1, int N2, int* S2) {
  *S2 = 1;
  if (orion_wgrad_splits(M, N1, N2) != 1) return 0;
  const long t1 = (N1 + 255) / 256, t2 = (N2 + 255) / 256, tiles = t1 * t2;
  if (tiles <= 256 || tiles % 256 == 0) return 0;
  const long head_rows = (tiles / 256) * 256 / t2;  // whole tile rows inside the whole rounds
  const long rem = tiles - head_rows * t2;
  if (head_rows < 1 || head_rows >= t1 || rem > 128) return 0;
  const int s2 = orion_wgrad_effective_splits(M, (int)(256 / rem));
  if (s2 < 2) return 0;
  *S2 = s2;
  return (int)head_rows * 256;
}

// number of k-chunks actually produced when S are requested (chunks are whole stages)
int orion_wgrad_effective_splits(int M, int S) {
  if (S < 1) S = 1;
  const int BK = wg_bk(M);
  const int chunk = ((M / BK + S - 1) / S) * BK;
  return chunk > 0 ? (M + chunk - 1) / chunk : 1;
}

// A (M x N1, ld lda), B (M x N2, ld ldb) bf16 -> slabs (S, N1, N2) fp32 when S > 1
// (caller folds them), else out (N1, N2; fp32 when out_f32, else bf16) scaled by *scale
// (nullable), added to the values already in out when accumulate != 0.  bt != 0: B is given
// transposed, (N2 x M, ld ldb) -- the NT operand of gemm16 (one ds_read_b128 per fragment
// instead of two transposing reads; M % 64 == 0).
int orion_wgrad(const void* A, long lda, const void* B, long ldb, int M, int N1, int N2, int S,
                float* slabs, void* out, const float* scale, int accumulate, int out_f32, int bt,
                hipStream_t st) {
  const int BK = wg_bk(M);
  if (M % BK || N1 % 8 || N2 % 8 || lda % 8 || ldb % 8 || N1 < 8 || N2 < 8) return -1;
  if (bt && BK != 64) return -1;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15) return -2;
  const int chunk = ((M / BK + S - 1) / S) * BK;
  const int Se = (M + chunk - 1) / chunk;
  if (Se != S) return -3;
  if (S > 1 && !slabs) return -4;
  const int t1 = (N1 + 255) / 256, t2 = (N2 + 255) / 256;
  const int ntiles = t1 * t2;
  const long lim = 0xFFFFFF00L;
  const bool fits = (long)chunk * lda * 2 < lim && (bt ? 256L * ldb * 2 : (long)chunk * ldb * 2) < lim;
  if (bt && !fits) return -1;
  if (BK == 64 && fits) {
    GemmArgs a{};
    a.X = (const bf16_t*)A;  // [M tokens][N1]: the k-major "X" operand, rows of out = N1
    a.ldx = lda;
    a.W = (const bf16_t*)B;  // [M tokens][N2], or (bt) [N2][M tokens]
    a.ldw = ldb;
    a.out = (bf16_t*)out;
    a.ldo = N2;
    a.M = N1;
    a.N = N2;
    a.K = M;
    a.tiles_n = t2;
    a.kchunk = chunk;
    a.ksplit = S;
    a.slabs = S > 1 ? slabs : nullptr;
    a.scale = scale;
    a.accumulate = accumulate;
    a.out_f32 = out_f32;
    return gemm16_wgrad(a, bt, st);
  }
  constexpr int lds = WG_NS * WG_KS * 16 * 128 * 4 * (int)sizeof(bf16_t);
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)wgrad_kernel<WG_KS, WG_NS, WG_WM>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
      return -5;
    attr = true;
  }
  wgrad_kernel<WG_KS, WG_NS, WG_WM><<<ntiles * S, WG_WM * 256, lds, st>>>(
      (const bf16_t*)A, lda, (const bf16_t*)B, ldb, M, N1, N2, t2, ntiles, chunk, S > 1 ? slabs : nullptr,
      out, scale, accumulate, out_f32);
  return (int)hipGetLastError();
}
