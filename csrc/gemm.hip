// Forward and input-gradient GEMMs of the linear layers for gfx950, with fused epilogues.
//
//   forward  (NT):  Y[m][n]  = sum_k X[m][k] W[n][k]          W stored [N][K] (nn.Linear)
//   dgrad    (NN):  dX[m][n] = sum_k dY[m][k] W[k][n]         W stored [K][N] (same tensor)
//
// Epilogues (fp32, before the single bf16 rounding of the output):
//   EPI_STORE      out = acc
//   EPI_BIAS       out = acc + bias[n]                                       (QKV projection)
//   EPI_BIAS_GELU  out = a = acc + bias[n], out2 = gelu_tanh(a)              (MLP c_fc)
//   EPI_GELU_BWD   out = acc * gelu_tanh'(pre[m][n])                         (MLP c_proj dgrad)
// The last two remove the separate bias+GELU forward and GELU backward HBM passes over
// the (tokens x 4C) activation: hipBLASLt has no AUX/BGRAD GELU epilogue kernels on gfx950
// (docs/PERFORMANCE.md), so this is where the fusion has to live.
//
// Structure (one 512-thread workgroup per 256 x 256 output tile, one per CU):
//   * "swapped" MFMA orientation: v_mfma_f32_32x32x16_bf16 with the W tile as the A operand
//     and the X tile as the B operand computes C^T; a lane then owns one output ROW m and
//     its registers walk 4-column runs of n, so the epilogue packs 8 consecutive bf16 per
//     lane after one v_permlane32_swap per register pair (16-byte stores, T21);
//   * 8 waves as 2 (n) x 4 (m), 128 x 64 outputs = 4 x 2 accumulators (128 registers) each;
//   * K in stages of 64: X as a [256][64] image (128-B rows) read by ds_read_b128; W as
//     the same (NT) or, for the k-major NN operand, as two [64][128] halves read by the
//     transposing ds_read_b64_tr_b16 (natural k order, so X needs no permutation); all
//     images XOR-swizzled (mfma_lds.h) with the swizzle applied to the per-lane SOURCE
//     address of the LDS-DMA fill;
//   * LDS-DMA (global_load_lds_dwordx4) into a 2-stage ring (128 KB): stage t+1 is issued
//     right after the barrier that retires stage t and lands under stage t's 32 MFMAs per
//     wave; fragment reads are inline asm (so the compiler does not drain the DMA before
//     them) double-buffered across the four 16-deep k steps;
//   * XCD-aware tile order: the tiles that share an X row panel are consecutive work ids,
//     and consecutive work ids run on one XCD (bijective remap), so the panel is read
//     from that XCD's L2.
#include "gemm_common.h"

namespace orion {

// wait until at most N LDS reads are outstanding, with the fragments as "+v" operands (no
// MFMA reading them can be scheduled before the wait)
template <int N, int TJ>
ORION_DEVICE void lds_wait_set(bf16x8 (&w)[4], bf16x8 (&x)[TJ]) {
  if constexpr (TJ == 2) {
    asm volatile("s_waitcnt lgkmcnt(%6)"
                 : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(x[0]), "+v"(x[1]) : "n"(N));
  } else {
    static_assert(TJ == 4, "TJ in {2, 4}");
    asm volatile("s_waitcnt lgkmcnt(%8)"
                 : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(x[0]), "+v"(x[1]),
                   "+v"(x[2]), "+v"(x[3])
                 : "n"(N));
  }
}

// K-stage depth BK and ring depth NS (LDS = NS * BK KB): {64, 2} or {32, 4}
template <int BK, int NS>
constexpr int gemm_lds() { return NS * 2 * 256 * BK * 2; }

// element offset of (row, col) in a [256][BK] operand image
template <int BK>
ORION_DEVICE int img_off(int row, int col) {
  if constexpr (BK == 64) return loff<64>(row, col);
  else return loff32(row, col);
}
template <int BK>
ORION_DEVICE int img_swz(int row) {
  if constexpr (BK == 64) return swz<64>(row);
  else return (row >> 2) & 3;
}

// WM = waves along m: 4 -> 8 waves of 128 (n) x 64 (m) outputs (2 waves per SIMD); 2 -> 4
// waves of 128 x 128 (one wave per SIMD, 256 accumulator registers in AGPRs: half the LDS
// fragment reads per MFMA).
template <bool WKM, int EPI, int BK, int NS, int WM = 4>
__global__ __launch_bounds__(128 * WM, 1) void gemm_kernel(GemmArgs g) {
  constexpr int NW = 2 * WM, TJ = 8 / WM;  // waves; 32-column m tiles per wave
  constexpr int IMG = 256 * BK, STAGE = 2 * IMG;
  constexpr int NR = (WKM ? 8 : 4) + TJ;  // LDS reads per fragment set (X TJ b128, W 4 b128 | 8 tr)
  constexpr int RPB = 1024 / (2 * BK);   // image rows per one-KB LDS-DMA block
  constexpr int CPR = BK / 8;            // 16-byte chunks per image row
  constexpr int XB = 256 / RPB / NW;     // blocks per wave per [256][BK] image
  constexpr int WB = (WKM ? BK / 2 : 256 / RPB) / NW;  // blocks per wave of the W image
  constexpr int PS = XB + WB;            // LDS-DMA instructions per stage per wave
  static_assert(XB >= 1 && WB >= 1, "stage blocks must divide over the waves");
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h32 = lane >> 5, l32 = lane & 31;
  const int wn = wv / WM, wm = wv % WM;

  // bijective XCD remap: blocks bid, bid + 8, ... share an XCD; give each XCD a contiguous
  // range of work ids (tiles of one X row panel are consecutive)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int mt = wid / g.tiles_n, nt = wid % g.tiles_n;
  const int m0 = mt * 256, n0 = nt * 256;
  const int nk = g.K / BK;

  // LDS-DMA fill in one-KB blocks (one wave-instruction each):
  //   [256][BK] image (X; W for NT): block = RPB rows; lane -> row RPB b + lane / CPR, LDS
  //   slot lane % CPR holds source chunk slot ^ img_swz(row).
  //   [BK][128] halves (W for NN): block = half b / (BK/4), 4 rows; lane -> row + lane/16,
  //   slot lane % 16 holds source chunk slot ^ swz<128>(row).
  // Rows / columns past M or N are clamped onto valid memory; their outputs are not stored.
  long gx[XB], gw[WB];
  int lx[XB], lw[WB];
#pragma unroll
  for (int i = 0; i < XB; ++i) {
    const int blk = wv * XB + i;
    const int row = RPB * blk + lane / CPR, slot = lane % CPR;
    const int ch = slot ^ img_swz<BK>(row);
    gx[i] = (long)min(m0 + row, g.M - 1) * g.ldx + 8 * ch;
    lx[i] = blk * 512;
  }
#pragma unroll
  for (int i = 0; i < WB; ++i) {
    const int blk = wv * WB + i;
    if constexpr (WKM) {
      const int half = blk / (BK / 4), rb = blk % (BK / 4);
      const int row = 4 * rb + (lane >> 4), slot = lane & 15;
      const int col = half * 128 + 8 * (slot ^ swz<128>(row));
      gw[i] = (long)row * g.ldw + min(n0 + col, g.N - 8);
      lw[i] = half * (BK * 128) + rb * 512;
    } else {
      const int row = RPB * blk + lane / CPR, slot = lane % CPR;
      gw[i] = (long)min(n0 + row, g.N - 1) * g.ldw + 8 * (slot ^ img_swz<BK>(row));
      lw[i] = blk * 512;
    }
  }
  auto issue_x = [&](int t, int i) {
    ORION_DASSERT((t + 1) * BK <= g.K && gx[i] / g.ldx < g.M);
    glds16(g.X + (long)t * BK + gx[i], smem + (t % NS) * STAGE + lx[i]);
  };
  auto issue_w = [&](int t, int i) {
    bf16_t* dst = smem + (t % NS) * STAGE + IMG + lw[i];
    if constexpr (WKM) glds16(g.W + (long)t * BK * g.ldw + gw[i], dst);
    else glds16(g.W + (long)t * BK + gw[i], dst);
  };
  auto issue = [&](int t) {
#pragma unroll
    for (int i = 0; i < XB; ++i) issue_x(t, i);
#pragma unroll
    for (int i = 0; i < WB; ++i) issue_w(t, i);
  };
  // LDS-DMA spread over the k16 steps of a stage (the TA takes ~32 cycles per 1-KB DMA
  // instruction; a burst of them blocks the issuing wave, so interleave with the MFMAs)
  constexpr int KSTEPS = BK / 16;
  auto issue_step = [&](int t, int s) {
#pragma unroll
    for (int i = 0; i < XB; ++i)
      if (i % KSTEPS == s) issue_x(t, i);
#pragma unroll
    for (int i = 0; i < WB; ++i)
      if (i % KSTEPS == s) issue_w(t, i);
  };

  f32x16 acc[4][TJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = zero16();

  const int pre = min(nk, NS - 1);
  for (int st = 0; st < pre; ++st) issue(st);
  for (int t = 0; t < nk; ++t) {
    // this wave's share of stage t has landed; stages t+1 .. t+NS-2 may stay in flight
    const int ahead = min(nk - 1 - t, NS - 2);
    if constexpr (NS >= 5) {
      if (ahead >= 3) wait_vm_exact<3 * PS>();
      else if (ahead == 2) wait_vm_exact<2 * PS>();
      else if (ahead == 1) wait_vm_exact<PS>();
      else wait_vm_exact<0>();
    } else if constexpr (NS == 4) {
      if (ahead >= 2) wait_vm_exact<2 * PS>();
      else if (ahead == 1) wait_vm_exact<PS>();
      else wait_vm_exact<0>();
    } else if constexpr (NS == 3) {
      if (ahead >= 1) wait_vm_exact<PS>();
      else wait_vm_exact<0>();
    } else {
      wait_vm_exact<0>();
    }
    asm volatile("s_barrier" ::: "memory");   // everyone's share landed; slot of t-1 is free
    const bool refill = t + NS - 1 < nk && !(g.flags & 1);
    if (refill && !(g.flags & 2)) issue(t + NS - 1);
    const bf16_t* Xs = smem + (t % NS) * STAGE;
    const bf16_t* Ws = Xs + IMG;
    bf16x8 wf[2][4], xf[2][TJ];
    auto fetch = [&](int s, int slot) {
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        xf[slot][j] = b128_read(Xs, img_off<BK>(wm * (32 * TJ) + j * 32 + l32, 16 * s + 8 * h32));
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (WKM)
          wf[slot][i] = tr_frag_asm(Ws + wn * (BK * 128), 16 * s + 8 * h32, i * 32, lane, 4);
        else
          wf[slot][i] = b128_read(Ws, img_off<BK>(wn * 128 + i * 32 + l32, 16 * s + 8 * h32));
      }
    };
    fetch(0, 0);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int cur = s & 1;
      if (refill && (g.flags & 2)) issue_step(t + NS - 1, s);
      if (s + 1 < BK / 16) {
        fetch(s + 1, cur ^ 1);
        lds_wait_set<NR>(wf[cur], xf[cur]);  // step s = the older set
      } else {
        lds_wait_set<0>(wf[cur], xf[cur]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = mfma32(wf[cur][i], xf[cur][j], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // epilogue: acc[i][j] = C^T tile; lane -> row m, register 4 g4 + e -> column
  // n = nb + 8 g4 + 4 h32 + e with nb the tile's first column
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int m = m0 + wm * (32 * TJ) + j * 32 + l32;
    const int mc = min(m, g.M - 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) gemm_epilogue_tile<EPI>(g, acc[i][j], m, mc, n0 + wn * 128 + i * 32, h32);
  }
}


// ---------------------------------------------------------------- ping-pong variant
// Same tile, operands, LDS images and epilogue as gemm_kernel, scheduled so that the two
// 4-wave groups (grp 0: waves 0-3 = n rows 0-127, grp 1: waves 4-7 = n rows 128-255; one
// wave of each group per SIMD) alternate roles every barrier: while one group issues its
// 16-MFMA cluster (one 32-deep k chunk: 2 x 4 x 2 v_mfma_f32_32x32x16_bf16), the other
// reads the fragments of its next chunk from LDS and issues the LDS-DMA of the next stage.
// grp 1 runs one barrier behind grp 0 (one extra s_barrier before its first chunk; grp 0
// adds one after its last).  Per wave, in its own time: L(c) | C(c) for chunks c = 0, 1, ...
// with a barrier after each; globally grp 0 runs L(c) in slot 2c and C(c) in 2c+1, grp 1
// one slot later.
// LDS hazards (2-stage ring, stage t = chunks 2t, 2t+1):
//   * WAR: stage t+1 is staged into the buffer of stage t-1 at the start of L(2t); the
//     last reader of stage t-1 is grp 1's L(2t-1) in slot 4t-1 and every L segment ends
//     with lgkmcnt(0) before its barrier, so those reads are complete;
//   * RAW: the first reader of stage t+1 is grp 0's L(2t+2) in slot 4t+4; each wave waits
//     vmcnt(0) for its own DMA before the barrier that closes slot 4t+3 (grp 0 after
//     C(2t+1), grp 1 after L(2t+1)).
template <bool WKM, int EPI>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(GemmArgs g) {
  constexpr int BK = 64, IMG = 256 * BK, STAGE = 2 * IMG;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform
  const int h32 = lane >> 5, l32 = lane & 31;
  const int grp = wv >> 2, wm = wv & 3;

  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int mt = wid / g.tiles_n, nt = wid % g.tiles_n;
  const int m0 = mt * 256, n0 = nt * 256;
  const int nk = g.K / BK;

  // LDS-DMA fill (as gemm_kernel with BK = 64): 4 X blocks and 4 W blocks per wave
  long gx[4], gw[4];
  int lx[4], lw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int blk = wv * 4 + i;
    const int row = 8 * blk + (lane >> 3), slot = lane & 7;
    const int ch = slot ^ swz<64>(row);
    gx[i] = (long)min(m0 + row, g.M - 1) * g.ldx + 8 * ch;
    lx[i] = blk * 512;
    if constexpr (WKM) {
      const int half = blk >> 4, rb = blk & 15;
      const int r4 = 4 * rb + (lane >> 4), s16 = lane & 15;
      const int col = half * 128 + 8 * (s16 ^ swz<128>(r4));
      gw[i] = (long)r4 * g.ldw + min(n0 + col, g.N - 8);
      lw[i] = half * (BK * 128) + rb * 512;
    } else {
      gw[i] = (long)min(n0 + row, g.N - 1) * g.ldw + 8 * ch;
      lw[i] = blk * 512;
    }
  }
  auto issue = [&](int t) {
    bf16_t* base = smem + (t & 1) * STAGE;
    const long kk = (long)t * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      glds16(g.X + kk + gx[i], base + lx[i]);
      if constexpr (WKM) glds16(g.W + kk * g.ldw + gw[i], base + IMG + lw[i]);
      else glds16(g.W + kk + gw[i], base + IMG + lw[i]);
    }
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();

  bf16x8 wf[2][4], xf[2][2];  // one 32-deep chunk: [k16 step][tile]
  auto load_chunk = [&](int c) {
    const bf16_t* Xs = smem + ((c >> 1) & 1) * STAGE;
    const bf16_t* Ws = Xs + IMG;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int kc = 32 * (c & 1) + 16 * s + 8 * h32;  // k column inside the stage
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (WKM)
          wf[s][i] = tr_frag_asm(Ws + grp * (BK * 128), kc, i * 32, lane, 4);
        else
          wf[s][i] = b128_read(Ws, loff<64>(grp * 128 + i * 32 + l32, kc));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) xf[s][j] = b128_read(Xs, loff<64>(wm * 64 + j * 32 + l32, kc));
    }
    // every fragment read retired before this segment's barrier (WAR for the next DMA)
    lds_wait_frags<0, 4>(wf[0], xf[0]);
    lds_wait_frags<0, 4>(wf[1], xf[1]);
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  issue(0);
  wait_vm_exact<0>();
  barrier();
  if (grp == 1) barrier();  // the stagger
  for (int c = 0; c < 2 * nk; ++c) {
    const int t = c >> 1;
    const bool even = (c & 1) == 0;
    if (even && t + 1 < nk && !(g.flags & 1)) issue(t + 1);
    load_chunk(c);
    if (!even && grp == 1 && t + 1 < nk) wait_vm_exact<0>();
    barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(wf[s][i], xf[s][j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    if (!even && grp == 0 && t + 1 < nk) wait_vm_exact<0>();
    barrier();
  }
  if (grp == 0) barrier();  // match grp 1's barrier count

  const int wn = grp;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = m0 + wm * 64 + j * 32 + l32;
    const int mc = min(m, g.M - 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nb = n0 + wn * 128 + i * 32;
      gemm_epilogue_tile<EPI>(g, acc[i][j], m, mc, nb, h32);
    }
  }
}

}  // namespace orion

using namespace orion;

// ORION_GEMM_CFG: 9 = the 16x16x32-MFMA phased kernel (csrc/gemm16.hip, default; round 3: 5-15 %
// faster than 7 on every GPT-2 / Llama shape measured), 7 = the 32x32x16 phased kernel
// (csrc/gemm_phased.hip; 8 = its 4-quadrant
// schedule), 0 = BK 64 x 2 stages, 1 = ping-pong, 2 = BK 32 x 4-stage ring,
// 3 = BK 32 x 5-stage ring (160 KB: three stages in flight), 4/5/6 = 4 waves of 128 x 128
// with BK 64 x 2 / BK 32 x 4 / BK 32 x 5 (docs/PERFORMANCE.md, "In-tree GEMM study").
static int gemm_cfg() {  // read per call: microbenchmarks switch variants in one process
  const char* e = getenv("ORION_GEMM_CFG");
  const int c = e ? atoi(e) : 9;
  return c < 0 || c > 9 ? 9 : c;
}

template <bool WKM, int EPI, int BK, int NS, int WM = 4>
static int gemm_launch_cfg(const GemmArgs& a, hipStream_t st) {
  static bool attr = false;
  constexpr int lds = gemm_lds<BK, NS>();
  if (!attr) {
    if (hipFuncSetAttribute((const void*)gemm_kernel<WKM, EPI, BK, NS, WM>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
      return -5;
    attr = true;
  }
  const int tiles_m = (a.M + 255) / 256;
  gemm_kernel<WKM, EPI, BK, NS, WM><<<tiles_m * a.tiles_n, 128 * WM, lds, st>>>(a);
  return (int)hipGetLastError();
}

template <bool WKM, int EPI>
static int gemm_launch_pp(const GemmArgs& a, hipStream_t st) {
  static bool attr = false;
  constexpr int lds = gemm_lds<64, 2>();
  if (!attr) {
    if (hipFuncSetAttribute((const void*)gemm_pp_kernel<WKM, EPI>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
      return -5;
    attr = true;
  }
  const int tiles_m = (a.M + 255) / 256;
  gemm_pp_kernel<WKM, EPI><<<tiles_m * a.tiles_n, 512, lds, st>>>(a);
  return (int)hipGetLastError();
}

template <bool WKM, int EPI>
static int gemm_launch(const GemmArgs& a, hipStream_t st) {
  switch (gemm_cfg()) {
    case 1: return gemm_launch_pp<WKM, EPI>(a, st);
    case 2: return gemm_launch_cfg<WKM, EPI, 32, 4>(a, st);
    case 3: return gemm_launch_cfg<WKM, EPI, 32, 5>(a, st);
    case 4: return gemm_launch_cfg<WKM, EPI, 64, 2, 2>(a, st);
    case 5: return gemm_launch_cfg<WKM, EPI, 32, 4, 2>(a, st);
    case 6: return gemm_launch_cfg<WKM, EPI, 32, 5, 2>(a, st);
    default: return gemm_launch_cfg<WKM, EPI, 64, 2>(a, st);
  }
}

// out[M][N] = X[M][K] . op(W) with op(W) = W^T for W [N][K] (wkm = 0) or W for W [K][N]
// (wkm = 1), epilogue `epi` (GemmEpi).  Requirements (else -1): K % 64 == 0, N % 8 == 0,
// N >= 8, 8-element aligned leading dims, 16-byte aligned base pointers.
int orion_colsum_bf16(const void* m, void* out, float* part, int rows, int C, int out_f32,
                      hipStream_t st);
int orion_colsum_partials2(const float* part, float* mid, void* out, int P, int C, int f32,
                           hipStream_t st);

// EPI_GELU_BWD with db: db[N] (fp32 when db_f32, else bf16) = column sums of the result (the
// bias gradient) through part (orion_gemm_colsum_scratch(M, N) floats): per-64-row partials
// from the phased kernel's epilogue, else a column-sum pass over out.
int orion_gemm_colsum_scratch(int M, int N) { return ((M + 63) / 64 + 32) * N; }

int orion_gemm(const void* X, long ldx, const void* W, long ldw, int M, int N, int K, int wkm,
               int epi, void* out, long ldo, const void* bias, void* out2, long ldo2,
               const void* pre, long ldp, hipStream_t st, void* db, int db_f32, float* part) {
  if (M < 1 || K < 64 || K % 64 || N % 8 || N < 8) return -1;
  if ((ldx | ldw | ldo) % 8) return -1;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) |
       reinterpret_cast<uintptr_t>(out)) & 15) return -2;
  if ((epi == EPI_BIAS || epi == EPI_BIAS_GELU) && !bias) return -3;
  if (epi == EPI_BIAS_GELU && (!out2 || ldo2 % 8 || (reinterpret_cast<uintptr_t>(out2) & 15))) return -3;
  if (epi == EPI_GELU_BWD && (!pre || ldp % 4)) return -3;
  if (db && (epi != EPI_GELU_BWD || !part || ldo != N)) return -3;
  GemmArgs a{(const bf16_t*)X, ldx, (const bf16_t*)W, ldw, (bf16_t*)out, ldo,
             (const bf16_t*)bias, (bf16_t*)out2, ldo2, (const bf16_t*)pre, ldp,
             M, N, K, (N + 255) / 256, 0};
  if (const char* e = getenv("ORION_GEMM_DIAG")) a.flags = atoi(e);
  if ((a.flags & 4) && epi == EPI_STORE) a.slabs = (float*)pre;  // slot stamps (diagnostic)
  const int cfg = gemm_cfg();
  if (cfg == 8) a.flags |= 16;  // phased kernel, SCHED 0 (8-MFMA quadrant phases)
  int rc;
  if (cfg == 9 && gemm16_ok(a, wkm) &&
      (epi != EPI_GELU_BWD || (ldp % 8 == 0 && !(reinterpret_cast<uintptr_t>(pre) & 15)))) {
    const int rows = (M + 63) / 64;
    if (db) a.colsum = part;
    rc = gemm16(a, wkm, epi, st);
    if (rc == 0 && db) rc = orion_colsum_partials2(part, part + (long)rows * N, db, rows, N, db_f32, st);
    return rc;
  }
  if ((cfg == 7 || cfg == 8 || cfg == 9) && gemm_phased_ok(a, wkm)) {
    const int rows = (M + 63) / 64;
    if (db) a.colsum = part;
    rc = gemm_phased(a, wkm, epi, st);
    if (rc == 0 && db) rc = orion_colsum_partials2(part, part + (long)rows * N, db, rows, N, db_f32, st);
    return rc;
  }
  switch (epi * 2 + (wkm ? 1 : 0)) {
    case EPI_STORE * 2 + 0: rc = gemm_launch<false, EPI_STORE>(a, st); break;
    case EPI_STORE * 2 + 1: rc = gemm_launch<true, EPI_STORE>(a, st); break;
    case EPI_BIAS * 2 + 0: rc = gemm_launch<false, EPI_BIAS>(a, st); break;
    case EPI_BIAS_GELU * 2 + 0: rc = gemm_launch<false, EPI_BIAS_GELU>(a, st); break;
    case EPI_GELU_BWD * 2 + 1: rc = gemm_launch<true, EPI_GELU_BWD>(a, st); break;
    default: return -4;
  }
  if (rc == 0 && db) rc = orion_colsum_bf16(out, db, part, M, N, db_f32, st);
  return rc;
}
