// Phase-interleaved linear-layer GEMM for gfx950 (forward NT and dgrad NN, fused epilogues):
// the same operands, tile and epilogue as csrc/gemm.hip, scheduled so that matrix-core
// work, LDS fragment reads and LDS-DMA staging overlap at a fine grain.
//
// Tile 256 (n) x 256 (m) per 512-thread workgroup, one workgroup per CU, K in 64-deep
// k-tiles.  Swapped MFMA orientation (W tile = A operand, X tile = B operand, C^T in the
// accumulators), 8 waves as 2 groups (grp = n half) x 4 (wm = 64 m rows): each wave owns
// 128 n x 64 m = 4 x 2 accumulators of v_mfma_f32_32x32x16_bf16.
//
// Phases.  A k-tile is 4 phases; phase q computes one quadrant of the wave's outputs with
// 8 MFMAs (256 matrix-core cycles):
//     q0: n-half 0 x m-tile 0   reads W half 0 (8 frags) + X m-tile 0 (4 frags)
//     q1: n-half 0 x m-tile 1   reads X m-tile 1
//     q2: n-half 1 x m-tile 0   reads W half 1
//     q3: n-half 1 x m-tile 1   (no reads)
// so every fragment register is rewritten at least two phases after its last MFMA use and
// the 96 fragment registers are read from LDS once per k-tile.  A phase is two barrier
// slots -- READ (fragment reads + this phase's LDS-DMA) and MMA (wait lgkmcnt(0), 8 MFMAs at
// raised priority) -- and group 1 runs one slot behind group 0, so on every SIMD (one wave
// of each group) one wave issues MFMAs while the other reads LDS and feeds the DMA.
//
// Staging.  A k-tile's operands are 4 pieces of 16 KB (128 rows x 64 k), named by the
// quadrant that first reads them: A = W rows of n-half 0 (both groups), B = X rows of m-tile
// 0 (all wm), C = X m-tile 1, D = W n-half 1.  Each phase stages ONE piece (each group its
// half, 2 buffer_load_dwordx4 ... lds per wave), so the texture path sees a steady 8 KB per
// slot instead of bursts.  Piece k of k-tile t is issued at phase 4t + {-6,-5,-4,-3}[k] and
// first read at 4t + {0,0,1,2}[k]: >= 5 phases (~10 slots) of latency cover, and its
// 2-buffer LDS slot was last read >= 2 phases earlier (each piece is read in one phase
// only).  Waits: after a wave's phase-P DMA is issued, s_waitcnt vmcnt(<loads of phases
// P-3..P>) retires everything the next phase reads, placed before the barrier that opens
// group 0's next READ slot (group 0: end of its MMA slot; group 1: end of its READ slot).
// Raw s_barrier throughout (a __syncthreads() would drain the DMA queue), all LDS in one
// dynamic array, fragment reads as inline asm with hand-counted lgkmcnt.
//
// Operand images (elements, per stage: X [256][64] then W): X and NT W as [256][64] with
// 128-byte rows, 16-byte chunk c of row r at c ^ swz<64>(r) (mfma_lds.h); NN W (k-major) as
// four [64 k][64 n] quarter images (group, n-half), read by ds_read_b64_tr_b16.  Rows /
// columns past M or N are clamped onto valid memory (their outputs are not stored).
#include "gemm_common.h"

namespace orion {

namespace {

constexpr int PH_BK = 64, PH_IMG = 256 * PH_BK, PH_STAGE = 2 * PH_IMG;
constexpr int PH_LDS_BYTES = 2 * PH_STAGE * 2;  // 128 KB (SCHED 0)
constexpr int PH2_X0 = 0, PH2_W0 = 3 * PH_IMG;   // SCHED 1: X images x3, then W images x2
constexpr int PH2_LDS_BYTES = 5 * PH_IMG * 2;    // 160 KB

ORION_DEVICE void ph_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// fragment reads retired; the fragments become "+v" operands so no MFMA using them can be
// scheduled before the wait
ORION_DEVICE void ph_wait_lds(bf16x8 (&w)[4], bf16x8 (&x)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]));
}
ORION_DEVICE void ph_wait_lds(bf16x8 (&x)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]));
}

}  // namespace

// STAMPS (diagnostic instantiation, ORION_GEMM_DIAG=4 with a stamp buffer, EPI_STORE only):
// workgroup 0 records s_memtime per wave at each slot boundary into g.slabs as u64
// [wave][1024] (scripts/gemm_stamps.py); no effect on results.
// SCHED 0 (flags & 16: ORION_GEMM_CFG / ORION_WGRAD_CFG = 8): four 8-MFMA quadrant phases per
// k-tile (2-deep ring of 64 KB stages).
// SCHED 1 (default, 2-3 % faster): two 16-MFMA phases per k-tile (n-half 0, n-half 1: half the barriers); the X
// images are triple-buffered (3 x 32 KB) so that both X pieces, read in the first phase, can
// be staged two phases earlier than the W pieces; W double-buffered (2 x 32 KB): 160 KB.
template <bool XKM, bool WKM, int EPI, bool STAMPS = false, int SCHED = 0>
__global__ __launch_bounds__(512, 1) void gemm_phased_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wv >> 2, wm = wv & 3;
  const int h32 = lane >> 5, l32 = lane & 31;

  // Work ids: with one workgroup per tile (gridDim = tiles) the bijective XCD remap of
  // gemm_kernel; persistent (gridDim = CUs, a multiple of 8, < tiles): XCD x owns the
  // contiguous work-id range [T x / 8, T (x+1) / 8) and its workgroups stride over it.  A work
  // id walks groups of GM m-tiles with the m-tile fastest, so the ~32 tiles an XCD runs at
  // once share GM X panels and ~32/GM W panels per k-tile in its L2.
  constexpr int GM = 4;
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7;
  const int tiles_m = (g.M + 255) >> 8, tiles = tiles_m * g.tiles_n, T = tiles * g.ksplit;
  int wid, wstride, wend;
  if (nwg >= T) {
    const int qq = nwg >> 3, rr = nwg & 7;
    wid = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
    wstride = T;
    wend = T;
  } else {
    wid = (int)((long)T * xcd / 8) + (bid >> 3);
    wstride = nwg >> 3;
    wend = (int)((long)T * (xcd + 1) / 8);
  }
  if (wid >= wend) return;
  // work id -> (k chunk kc, tile): the tiles of one k chunk are consecutive work ids
  auto tile_of = [&](int w, int& m0, int& n0, int& kc) {
    kc = w / tiles;
    w -= kc * tiles;
    const int grp_sz = GM * g.tiles_n, gidx = w / grp_sz, first_m = gidx * GM;
    const int gm = min(tiles_m - first_m, GM), in = w - gidx * grp_sz;
    m0 = (first_m + in % gm) * 256;
    n0 = (in / gm) * 256;
  };
  int m0, n0, kc;
  tile_of(wid, m0, n0, kc);
  int nk;  // k-tiles of the current work item

  // operand buffer resources of the current work item, based at its k chunk (so 32-bit
  // offsets suffice for any chunk < 4 GB), and bytes per k-tile
  __amdgpu_buffer_rsrc_t rx, rw;
  const unsigned xstep = XKM ? (unsigned)(PH_BK * g.ldx * 2) : PH_BK * 2;
  const unsigned wstep = WKM ? (unsigned)(PH_BK * g.ldw * 2) : PH_BK * 2;

  // LDS-DMA: piece p (0 A, 1 B, 2 C, 3 D), this wave's blocks e = 0, 1 of its group's 8 (one
  // block = 8 image rows x 128 B = one wave instruction, lane -> row lane / 8, chunk lane % 8)
  unsigned vo[4][2];
  int ld[4][2];
  const int lr = lane >> 3, slot = lane & 7;
  auto set_tile = [&](int m0, int n0, int kc) {
    const int k0 = kc * g.kchunk, kr = min(g.kchunk, g.K - k0);
    nk = kr / PH_BK;
    if constexpr (XKM) rx = make_rsrc(g.X + (long)k0 * g.ldx, (unsigned)((long)kr * g.ldx * 2));
    else rx = make_rsrc(g.X + k0, (unsigned)(((long)g.M * g.ldx - k0) * 2));
    if constexpr (WKM) rw = make_rsrc(g.W + (long)k0 * g.ldw, (unsigned)((long)kr * g.ldw * 2));
    else rw = make_rsrc(g.W + k0, (unsigned)(((long)g.N * g.ldw - k0) * 2));
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int b = 2 * wm + e;  // 0..7
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {  // X: B (m-tile 0 rows), C (m-tile 1 rows)
        if constexpr (XKM) {
          // [64 k][32 m] sub-image (jj, wm'), 64-byte rows, unswizzled; block = 16 k rows
          const int wmp = 2 * grp + (b >> 2), kr0 = (b & 3) * 16, k = kr0 + (lane >> 2);
          const int m = m0 + wmp * 64 + jj * 32 + 8 * (lane & 3);
          vo[1 + jj][e] = (unsigned)(((long)k * g.ldx + min(m, g.M - 8)) * 2);
          ld[1 + jj][e] = (jj * 4 + wmp) * 2048 + kr0 * 32;
        } else {
          const int row0 = (2 * grp + (b >> 2)) * 64 + jj * 32 + (b & 3) * 8, row = row0 + lr;
          const int ch = slot ^ swz<64>(row);
          vo[1 + jj][e] = (unsigned)(((long)min(m0 + row, g.M - 1) * g.ldx + 8 * ch) * 2);
          ld[1 + jj][e] = row0 * 64;
        }
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {  // W: A (n-half 0), D (n-half 1) of this group
        const int p = hh ? 3 : 0;
        if constexpr (WKM) {
          const int kr0 = b * 8, kr = kr0 + lr;
          const int col = n0 + grp * 128 + hh * 64 + 8 * (slot ^ swz<64>(kr));
          vo[p][e] = (unsigned)(((long)kr * g.ldw + min(col, g.N - 8)) * 2);
          ld[p][e] = (2 * grp + hh) * 4096 + kr0 * 64;
        } else {
          const int row0 = grp * 128 + hh * 64 + b * 8, row = row0 + lr;
          const int ch = slot ^ swz<64>(row);
          vo[p][e] = (unsigned)(((long)min(n0 + row, g.N - 1) * g.ldw + 8 * ch) * 2);
          ld[p][e] = row0 * 64;
        }
      }
    }
  };
  set_tile(m0, n0, kc);
  // LDS images of k-tile t
  auto ximg = [&](int t) -> bf16_t* {
    if constexpr (SCHED == 1) return smem + PH2_X0 + (t % 3) * PH_IMG;
    else return smem + (t & 1) * PH_STAGE;
  };
  auto wimg = [&](int t) -> bf16_t* {
    if constexpr (SCHED == 1) return smem + PH2_W0 + (t & 1) * PH_IMG;
    else return smem + (t & 1) * PH_STAGE + PH_IMG;
  };
  auto issue = [&](int p, int t) {
    const bool isx = p == 1 || p == 2;
    bf16_t* base = isx ? ximg(t) : wimg(t);
    const unsigned so = (unsigned)t * (isx ? xstep : wstep);
    ORION_DASSERT(t < nk);
#pragma unroll
    for (int e = 0; e < 2; ++e) blds16(isx ? rx : rw, vo[p][e], so, base + ld[p][e]);
  };

  f32x16 acc[4][2];
  bf16x8 W0[2][4], W1[2][4], X0[4], X1[4];  // [n-tile][k16 step], [k16 step]

  // per-lane element offsets inside a [..][64] image: row l32 of a 32-row tile, k16 step s
  int ko[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) ko[s] = loff<64>(l32, 16 * s + 8 * h32);
  auto read_x = [&](bf16x8 (&x)[4], const bf16_t* Xs, int j) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if constexpr (XKM) x[s] = tr_frag_asm_lin32(Xs + (j * 4 + wm) * 2048, 16 * s + 8 * h32, lane, 4);
      else x[s] = b128_read(Xs + (wm * 64 + j * 32) * 64, ko[s]);
    }
  };
  auto read_w = [&](bf16x8 (&w)[4], const bf16_t* Ws, int h, int i) {  // n-tile i of n-half h
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if constexpr (WKM)
        w[s] = tr_frag_asm<64>(Ws + (2 * grp + h) * 4096, 16 * s + 8 * h32, i * 32, lane, 4);
      else
        w[s] = b128_read(Ws + (grp * 128 + h * 64 + i * 32) * 64, ko[s]);
    }
  };
  int nstamp = 0;
  auto stamp = [&] {
    if constexpr (STAMPS) {
      if (blockIdx.x == 0 && lane == 0 && nstamp < 1024)
        reinterpret_cast<unsigned long*>(g.slabs)[wv * 1024 + nstamp] = __builtin_amdgcn_s_memtime();
      ++nstamp;
    }
  };
  auto mma = [&](bf16x8 (&w)[2][4], bf16x8 (&x)[4], int i0, int j) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i0 + i][j] = mfma32(w[i][s], x[s], acc[i0 + i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  // One phase of k-tile t: quadrant Q, stage its piece if ISSUE, then leave VMN loads in
  // flight (everything the next phase reads has landed).  All compile-time: no branches in
  // the slot code.
  auto phase = [&](auto Qc, auto ISSUEc, auto VMNc, int t) {
    constexpr int Q = decltype(Qc)::value, VMN = decltype(VMNc)::value;
    constexpr bool ISSUE = decltype(ISSUEc)::value;
    const bf16_t* Xs = ximg(t);
    const bf16_t* Ws = wimg(t);
    // ---- READ slot
    stamp();  // R: slot start (after the barrier)
    if constexpr (Q == 0) {
      read_w(W0[0], Ws, 0, 0);
      read_w(W0[1], Ws, 0, 1);
      read_x(X0, Xs, 0);
    } else if constexpr (Q == 1) {
      read_x(X1, Xs, 1);
    } else if constexpr (Q == 2) {
      read_w(W1[0], Ws, 1, 0);
      read_w(W1[1], Ws, 1, 1);
    }
    if constexpr (ISSUE) {  // q0: C(t+1), q1: D(t+1), q2: A(t+2), q3: B(t+2)
      if constexpr (Q == 0) issue(2, t + 1);
      else if constexpr (Q == 1) issue(3, t + 1);
      else if constexpr (Q == 2) issue(0, t + 2);
      else issue(1, t + 2);
    }
    wait_vm_exact<VMN>();
    ph_barrier();
    // ---- MMA slot
    if constexpr (Q == 0) {
      ph_wait_lds(W0[0], X0);
      ph_wait_lds(W0[1]);
      __builtin_amdgcn_sched_barrier(0);
      stamp();  // S: fragments landed, MFMAs start
      mma(W0, X0, 0, 0);
    } else if constexpr (Q == 1) {
      ph_wait_lds(X1);
      __builtin_amdgcn_sched_barrier(0);
      stamp();
      mma(W0, X1, 0, 1);
    } else if constexpr (Q == 2) {
      ph_wait_lds(W1[0], W1[1]);
      __builtin_amdgcn_sched_barrier(0);
      stamp();
      mma(W1, X0, 2, 0);
    } else {
      __builtin_amdgcn_sched_barrier(0);
      stamp();
      mma(W1, X1, 2, 1);
    }
    stamp();  // E: MFMAs issued
    ph_barrier();
  };
  // SCHED 1: phase H of k-tile t: READ slot = this phase's fragments (H 0: W n-half 0 and all
  // of X, 16; H 1: W n-half 1, 8) + its pieces (H 0: A(t+1), B(t+2); H 1: D(t+1), C(t+2)),
  // then VMN loads left in flight (this phase's: every older one has landed, and each piece
  // is read >= 2 phases after it was issued); MMA slot = 16 MFMAs on 4 accumulators per step.
  // X registers are rewritten one MMA slot after their last use: an MFMA has read its A/B
  // operands once issued, and every MFMA of the slot is issued before its closing barrier.
  auto phase2 = [&](auto Hc, auto ISWc, auto ISXc, auto VMNc, int t) {
    constexpr int H = decltype(Hc)::value, VMN = decltype(VMNc)::value;
    constexpr bool ISW = decltype(ISWc)::value, ISX = decltype(ISXc)::value;
    const bf16_t* Xs = ximg(t);
    const bf16_t* Ws = wimg(t);
    stamp();
    if constexpr (H == 0) {
      read_w(W0[0], Ws, 0, 0);
      read_w(W0[1], Ws, 0, 1);
      read_x(X0, Xs, 0);
      read_x(X1, Xs, 1);
      if constexpr (ISW) issue(0, t + 1);
      if constexpr (ISX) issue(1, t + 2);
    } else {
      read_w(W1[0], Ws, 1, 0);
      read_w(W1[1], Ws, 1, 1);
      if constexpr (ISW) issue(3, t + 1);
      if constexpr (ISX) issue(2, t + 2);
    }
    wait_vm_exact<VMN>();
    ph_barrier();
    if constexpr (H == 0) {
      ph_wait_lds(W0[0], X0);
      ph_wait_lds(W0[1], X1);
    } else {
      ph_wait_lds(W1[0], W1[1]);
    }
    __builtin_amdgcn_sched_barrier(0);
    stamp();
    bf16x8 (&w)[2][4] = H == 0 ? W0 : W1;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        acc[2 * H + i][0] = mfma32(w[i][s], X0[s], acc[2 * H + i][0]);
        acc[2 * H + i][1] = mfma32(w[i][s], X1[s], acc[2 * H + i][1]);
      }
    __builtin_amdgcn_s_setprio(0);
    stamp();
    ph_barrier();
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  using I4 = std::integral_constant<int, 4>;
  using I6 = std::integral_constant<int, 6>;
  using I8 = std::integral_constant<int, 8>;
  using Y = std::true_type;
  using N = std::false_type;

  // prologue: the pieces of phases -6 .. -1 (A0 B0 C0 D0 A1 B1); phase 0 needs A0 and B0
  auto prologue = [&] {
    if constexpr (SCHED == 1) {  // B0 C0 A0 D0 B1 C1: phase 0 needs the first three
      issue(1, 0);
      issue(2, 0);
      issue(0, 0);
      issue(3, 0);
      if (nk > 1) {
        issue(1, 1);
        issue(2, 1);
      }
    } else {
      issue(0, 0);
      issue(1, 0);
      issue(2, 0);
      issue(3, 0);
      if (nk > 1) {
        issue(0, 1);
        issue(1, 1);
      }
    }
  };
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(g.out, (unsigned)((long)g.M * g.ldo * 2));
  const __amdgpu_buffer_rsrc_t ro2 =
      make_rsrc(EPI == EPI_BIAS_GELU ? g.out2 : g.out, (unsigned)((long)g.M * (EPI == EPI_BIAS_GELU ? g.ldo2 : g.ldo) * 2));
  constexpr int STORES = EPI == EPI_BIAS_GELU ? 32 : 16;  // buffer stores per wave per tile
  const float wsc = (EPI == EPI_WGRAD && g.ksplit == 1 && g.scale) ? *g.scale : 1.f;

  prologue();
  bool first = true;
  while (true) {
    // A0 and B0 landed: 8 later prologue loads (4 if nk = 1) may be in flight, plus the
    // previous tile's STORES epilogue stores issued after them (vmcnt retires in order)
    constexpr int PRO_LATE = SCHED == 1 ? 6 : 8;  // prologue loads after the first phase's
    if (first || EPI == EPI_WGRAD) {  // (EPI_WGRAD's stores are not counted: wait for them)
      if (nk > 1) wait_vm_exact<PRO_LATE>();
      else wait_vm_exact<PRO_LATE - 4>();
    } else {
      if (nk > 1) wait_vm_exact<PRO_LATE + STORES>();
      else wait_vm_exact<PRO_LATE - 4 + STORES>();
    }
    first = false;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = zero16();
    ph_barrier();
    if (grp == 1) ph_barrier();  // the stagger: group 1 runs one slot behind

    // piece issues run through phase 4 nk - 7; after phase P a wave leaves the loads of
    // phases P-3 .. P in flight (8 while every phase issues, fewer in the tail)
    int t = 0;
    if constexpr (SCHED == 1) {
      for (; t < nk - 2; ++t) {
        phase2(I0(), Y(), Y(), I4(), t);
        phase2(I1(), Y(), Y(), I4(), t);
      }
      if (nk >= 2) {  // t = nk - 2: A, D of k-tile nk - 1
        phase2(I0(), Y(), N(), I2(), t);
        phase2(I1(), Y(), N(), I2(), t);
        ++t;
      }
      phase2(I0(), N(), N(), I0(), t);
      phase2(I1(), N(), N(), I0(), t);
    } else {
    for (; t < nk - 2; ++t) {
      phase(I0(), Y(), I8(), t);
      phase(I1(), Y(), I8(), t);
      phase(I2(), Y(), I8(), t);
      phase(I3(), Y(), I8(), t);
    }
    if (nk >= 2) {  // t = nk - 2: the last two pieces (C, D of k-tile nk - 1)
      phase(I0(), Y(), I8(), t);
      phase(I1(), Y(), I8(), t);
      phase(I2(), N(), I6(), t);
      phase(I3(), N(), I4(), t);
      ++t;
    }
    phase(I0(), N(), I2(), t);  // t = nk - 1 (for nk = 1: C0, D0 in flight after the prologue)
    phase(I1(), N(), I0(), t);
    phase(I2(), N(), I0(), t);
    phase(I3(), N(), I0(), t);
    }
    if (grp == 0) ph_barrier();  // match group 1's barrier count: every LDS read is done

    // next tile's prologue DMA first, then this tile's epilogue: the loads land while the
    // epilogue runs and its stores drain under the next tile's first phases
    const int cm0 = m0, cn0 = n0, ckc = kc;
    wid += wstride;
    const bool more = wid < wend;
    if (more) {
      tile_of(wid, m0, n0, kc);
      set_tile(m0, n0, kc);
      prologue();
    }
    if constexpr (EPI == EPI_WGRAD) {
      // fp32 partial tile into slab ckc, or the final gradient (fp32 arena or bf16, scaled,
      // optionally accumulated); lane = output row m, 4 consecutive columns per store
      float* slab = g.ksplit > 1 ? g.slabs + (long)ckc * g.M * g.N : nullptr;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = cm0 + wm * 64 + j * 32 + l32;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const int n = cn0 + grp * 128 + i * 32 + 8 * g4 + 4 * h32;
            if (m < g.M && n < g.N) {
              const long o = (long)m * g.N + n;
              f32x4 v;
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * g4 + e];
              if (slab) {
                *reinterpret_cast<f32x4*>(slab + o) = v;
              } else if (g.out_f32) {
                f32x4* dst = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(g.out) + o);
                v = v * wsc;
                if (g.accumulate) v += *dst;
                *dst = v;
              } else {
                bf16x4* dst = reinterpret_cast<bf16x4*>(g.out + o);
                bf16x4 r, prev;
                if (g.accumulate) prev = *dst;
#pragma unroll
                for (int e = 0; e < 4; ++e) r[e] = f2bf(v[e] * wsc + (g.accumulate ? bf2f(prev[e]) : 0.f));
                *dst = r;
              }
            }
          }
      }
      if (!more) break;
      continue;
    }
    constexpr bool CS = EPI == EPI_GELU_BWD;  // column sums of the result (bias gradient)
    const int mb = cm0 + wm * 64;              // this wave's 64-row block
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int nb = cn0 + grp * 128 + i * 32;
      float cs[CS ? 16 : 1];  // register r of acc[i][.]: this lane's sum over j
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int m = mb + j * 32 + l32;
        const int mc = min(m, g.M - 1);
        auto put = [&](const unsigned (&pk)[4][2], __amdgpu_buffer_rsrc_t r, long ld) {
#pragma unroll
          for (int pr = 0; pr < 2; ++pr) {
            const int n = nb + 16 * pr + 8 * h32;
            // always issued (the vmcnt count above relies on it); out-of-range lanes get an
            // offset past the buffer's end, which the hardware drops
            const bool ok = m < g.M && n < g.N && !(g.flags & 8);
            const unsigned off = ok ? (unsigned)(((long)m * ld + n) * 2) : 0xFFFFFFF0u;
            const uint4 w = gemm_epi_swap(pk, pr);
            u32x4 v;
            v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
            __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
          }
        };
        unsigned pk[4][2];
        if constexpr (CS) {
          float v[16];
          gemm_epi_values<EPI>(g, acc[i][j], mc, nb, h32, pk, v);
          const float keep = m < g.M ? 1.f : 0.f;  // rows past M repeat row M - 1
#pragma unroll
          for (int r = 0; r < 16; ++r) cs[r] = j ? cs[r] + keep * v[r] : keep * v[r];
        } else {
          gemm_epi_values<EPI>(g, acc[i][j], mc, nb, h32, pk);
        }
        put(pk, ro, g.ldo);
        if constexpr (EPI == EPI_BIAS_GELU) {
          gemm_epi_values<EPI, true>(g, acc[i][j], mc, nb, h32, pk);
          put(pk, ro2, g.ldo2);
        }
      }
      if constexpr (CS) {
        if (g.colsum) {
          // sum over the 32 lanes of each half (same columns n, rows m = lane): four halving
          // exchange steps (at offset o a lane keeps the half of its live values selected by
          // lane bit o and adds its partner's copy of it), then one full add with lane ^ 1;
          // lane l32 ends with register r = l32 / 2
          auto step = [&](auto Oc) {
            constexpr int o = decltype(Oc)::value, half = o / 2;
            const bool up = (l32 & o) != 0;
#pragma unroll
            for (int k = 0; k < half; ++k) {
              const float send = up ? cs[k] : cs[half + k];
              const float keep = up ? cs[half + k] : cs[k];
              cs[k] = keep + __shfl_xor(send, o);
            }
          };
          step(std::integral_constant<int, 16>());
          step(std::integral_constant<int, 8>());
          step(std::integral_constant<int, 4>());
          step(std::integral_constant<int, 2>());
          const float tot = cs[0] + __shfl_xor(cs[0], 1);
          const int r = l32 >> 1;
          const int n = nb + (r & 3) + 8 * (r >> 2) + 4 * h32;
          if (!(l32 & 1) && mb < g.M && n < g.N) g.colsum[(long)(mb / 64) * g.N + n] = tot;
        }
      }
    }
    if (!more) break;
  }
}

template <bool XKM, bool WKM, int EPI, bool STAMPS, int SCHED>
static int gemm_phased_launch_s(const GemmArgs& a, hipStream_t st) {
  constexpr int lds = SCHED == 1 ? PH2_LDS_BYTES : PH_LDS_BYTES;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)gemm_phased_kernel<XKM, WKM, EPI, STAMPS, SCHED>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
      return -5;
    attr = true;
  }
  static int ncu = 0;
  if (!ncu) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return -5;
    ncu = n >= 8 ? n & ~7 : 1 << 30;  // persistent grid: a multiple of 8 (one per XCD slot)
  }
  const long work = (long)((a.M + 255) / 256) * a.tiles_n * a.ksplit;
  // One workgroup per work item by default: the hardware dispatcher balances the tiles (also
  // around co-running RCCL kernels, which a static persistent split cannot), and it measured
  // equal (weight gradients) to 1-8 % faster (layer shapes) than the persistent walk, which
  // ORION_GEMM_PERSIST=1 selects (grid = CUs, next tile staged under the epilogue).
  static const bool persist = getenv("ORION_GEMM_PERSIST") && atoi(getenv("ORION_GEMM_PERSIST")) != 0;
  const int grid = (int)(work < ncu || !persist ? work : ncu);
  gemm_phased_kernel<XKM, WKM, EPI, STAMPS, SCHED><<<grid, 512, lds, st>>>(a);
  return (int)hipGetLastError();
}

template <bool XKM, bool WKM, int EPI>
static int gemm_phased_launch(const GemmArgs& a, hipStream_t st) {
  if constexpr (!XKM && EPI == EPI_STORE) {
    if ((a.flags & 4) && a.slabs) {
      if (a.flags & 16) return gemm_phased_launch_s<XKM, WKM, EPI, true, 0>(a, st);
      return gemm_phased_launch_s<XKM, WKM, EPI, true, 1>(a, st);
    }
  }
  if (a.flags & 16) return gemm_phased_launch_s<XKM, WKM, EPI, false, 0>(a, st);
  return gemm_phased_launch_s<XKM, WKM, EPI, false, 1>(a, st);
}

// Requirements beyond orion_gemm's: every operand and output byte offset fits in 32 bits
// (buffer addressing), below the out-of-range marker of the epilogue stores.
bool gemm_phased_ok(const GemmArgs& a, int wkm) {
  const long lim = 0xFFFFFF00L;
  const long xb = (long)a.M * a.ldx * 2, wb = (long)(wkm ? a.K : a.N) * a.ldw * 2;
  const long ob = (long)a.M * a.ldo * 2, o2 = a.out2 ? (long)a.M * a.ldo2 * 2 : 0;
  return xb < lim && wb < lim && ob < lim && o2 < lim;
}

int gemm_phased_wgrad(const GemmArgs& a, hipStream_t st) {
  return gemm_phased_launch<true, true, EPI_WGRAD>(a, st);
}

int gemm_phased(const GemmArgs& a0, int wkm, int epi, hipStream_t st) {
  GemmArgs a = a0;
  a.kchunk = a.K;
  a.ksplit = 1;
  switch (epi * 2 + (wkm ? 1 : 0)) {
    case EPI_STORE * 2 + 0: return gemm_phased_launch<false, false, EPI_STORE>(a, st);
    case EPI_STORE * 2 + 1: return gemm_phased_launch<false, true, EPI_STORE>(a, st);
    case EPI_BIAS * 2 + 0: return gemm_phased_launch<false, false, EPI_BIAS>(a, st);
    case EPI_BIAS_GELU * 2 + 0: return gemm_phased_launch<false, false, EPI_BIAS_GELU>(a, st);
    case EPI_GELU_BWD * 2 + 1: return gemm_phased_launch<false, true, EPI_GELU_BWD>(a, st);
    default: return -4;
  }
}

}  // namespace orion
