// Phase-interleaved linear-layer GEMM on v_mfma_f32_16x16x32_bf16 (gfx950): forward (NT),
// input gradient (NN) and weight gradient (k-major x k-major, split-K), fused epilogues.
// Persistent: one workgroup per CU walks a list of work items with ONE continuous LDS-DMA
// stream across them.
//
// On random operands the chip holds a higher clock on the 16x16x32 shape than on 32x32x16 at
// equal cycles per FLOP (MI355X_MICROARCH.md, DVFS give-back item 7: ~1.12-1.15x FLOP/s in
// LDS-fed loops).
//
// Tile 256 (n) x 256 (m) per 512-thread workgroup, K in 64-deep k-tiles.  Swapped
// orientation: the W tile is the A operand (rows n), the X tile the B operand (columns m),
// the accumulators hold C^T.  8 waves = 2 groups (grp = n half of 128) x 4 (wm = 64 m rows);
// a wave owns 128 n x 64 m = 8 x 4 accumulators of 16 x 16.
//
// Schedule (per k-tile, two phases H = 0, 1; group 1 runs one barrier slot behind group 0, so
// on every SIMD one wave issues MFMAs while the other reads LDS and feeds the DMA):
//   READ slot of phase H: fragment reads (H 0: W n-half 0 and all of X, 16 fragments; H 1:
//     W n-half 1, 8) + this phase's LDS-DMA pieces, then s_waitcnt vmcnt(<this phase's>);
//   MMA slot: wait lgkmcnt(0), 32 MFMAs (4 n-tiles x 4 m-tiles x 2 k-steps: 512 cycles).
// Pieces (16 KB each, 2 buffer_load_dwordx4 ... lds per wave): A = W n-half 0, D = W n-half 1,
// B / C = the two halves of the X image; A(s+1), B(s+2) issued in phase (s, 0), D(s+1), C(s+2)
// in phase (s, 1).  X images triple-buffered, W double-buffered: 160 KB of LDS.
//
// Work walk (round 4).  A per-CU timeline of the one-workgroup-per-item launch at K = 768
// (scripts/gemm16_timeline.py, profiles/gemm16/timeline_r04.txt) put 10-13 % of every CU's
// time in the prologue (the first pieces' HBM latency, nothing to overlap it with), 15-18 %
// in the epilogue and 3 % in workgroup dispatch.  Here the grid is at most one workgroup per
// CU and s counts k-tiles over the workgroup's whole item list: the pieces of the next item's
// first k-tiles are issued during the current item's last ones (the W stream runs one k-tile
// ahead of the MFMAs, the X stream two), so only the first item pays a prologue, and the
// epilogue of item j overlaps the DMA of item j + 1.  Items of one XCD: the blocks dealt to
// an XCD (b % 8) share a contiguous range of work ids and walk it with stride (blocks on
// that XCD), so the ~32 items an XCD runs at once stay neighbours in the grouped order (L2).
//
// LDS images, all lane-linear LDS-DMA destinations with the swizzle on the SOURCE address:
//   NT operand ([rows][64 k], 128-byte rows): 16-byte chunk c of row r at c ^ ((r >> 1) & 7);
//     the 16x16x32 fragment (row l & 15, k chunk 4 s + (l >> 4)) is one ds_read_b128, and the
//     four lane groups of the instruction hit 16 distinct bank slots;
//   k-major operand ([64 k][64 cols] per wave image, 128-byte rows): 32-byte segment s of row
//     k at s ^ ((k >> 1 & 1) | (k >> 3 & 1) << 1); the fragment (col l & 15, k 8 (l >> 4) + j)
//     is two ds_read_b64_tr_b16 (4 k rows x 16 cols per 16-lane group), conflict-free.
// Rows / columns past M or N are clamped onto valid memory; their outputs are not stored.
//
// Epilogue: a v_permlane16_swap per accumulator register pair of adjacent n-tiles gives every
// lane 8 consecutive n of one output row (fp32), so bias / GELU / GELU' read their operands
// and write the result as 16-byte row pieces; fp32 weight gradients store 16 bytes per
// register quadruple without a swap.
#include "gemm_common.h"

namespace orion {

namespace {

constexpr int G_BK = 64, G_IMG = 256 * G_BK;                 // bf16 elements per image
constexpr int G_X0 = 0, G_W0 = 3 * G_IMG, G_LDS = 5 * G_IMG * 2;  // 160 KB

ORION_DEVICE f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// one work item: output tile (m0, n0) and k chunk kc (split-K weight gradients)
struct G16Item {
  int m0, n0, kc, k0, kr, nk, rows_m, rows_n;
};

ORION_DEVICE G16Item g16_decode(const GemmArgs& g, int w) {
  // k chunk, then groups of GM m-tiles with the m-tile fastest (the ~32 tiles an XCD runs at
  // once share GM X panels and ~32 / GM W panels in its L2); flags bits 8-15 override GM
  // (diagnostic sweep)
  const int GM = (g.flags >> 8) & 0xFF ? (g.flags >> 8) & 0xFF : 4;
  const int tiles_m = (g.M + 255) >> 8, tiles = tiles_m * g.tiles_n;
  G16Item it;
  it.kc = w / tiles;
  w -= it.kc * tiles;
  const int grp_sz = GM * g.tiles_n, gidx = w / grp_sz, first_m = gidx * GM;
  const int gm = min(tiles_m - first_m, GM), in = w - gidx * grp_sz;
  it.m0 = (first_m + in % gm) * 256;
  it.n0 = (in / gm) * 256;
  it.k0 = it.kc * g.kchunk;
  it.kr = min(g.kchunk, g.K - it.k0);
  it.nk = it.kr / G_BK;
  it.rows_m = min(g.M - it.m0, 256);
  it.rows_n = min(g.N - it.n0, 256);
  return it;
}

}  // namespace

#ifndef G16_PRE_NT
#define G16_PRE_NT 1  // GPT-2 step: the fc2 / attn-proj forwards that read the GELU output next 166 -> 156 us (profiles/ab/gemm16_pre_nt_r04.log)
#endif
// Epilogue store shape (round 5).  Each lane holds 16 bytes (8 consecutive n) of one row after
// the permlane16_swap, so a plain store instruction covers 16 rows x 64 B.  G16_WIDE_ST = 1:
// a DPP row_ror:8 exchange between the packed results of two adjacent column pairs makes it
// 8 rows x 128 B (whole 128-byte lines): one store instruction touches half as many rows.
// Microbenchmark (scripts/micro/store_overlap.hip, profiles/micro_store_pattern_r05.log): with
// two workgroups per CU streaming LDS-DMA beside the stores, 16 x 64 B cost +0.14 ms over
// no stores, 8 x 128 B +0.09, 1 x 1 KB +0.03.
#ifndef G16_WIDE_ST
#define G16_WIDE_ST 1
#endif
// cache-policy bits of the second output (GELU activation / dup) and of plain outputs: nt (2).
// Same box, 2 rounds each (profiles/ab/gemm16_wide_nt_r05.log): LM-head forward 5.39-5.43 ms
// (16 x 64 B stores) -> 5.03 (8 x 128 B) -> 4.28-4.30 (8 x 128 B, nt; hipBLASLt 3.86); GPT-2
// step 1,119.9-1,124.0k -> 1,126.6-129.0k -> 1,136.1-1,137.2k tok/s.
#ifndef G16_ST_AUX
#define G16_ST_AUX 2
#endif
#ifndef G16_ST2_AUX
#define G16_ST2_AUX G16_ST_AUX  // the second output (GELU activation / SwiGLU dup)
#endif
// diagnostic: G16_DIAG_GELU=0 replaces GELU / GELU' by the identity (same loads and stores)
// to price the epilogue's transcendental arithmetic
#ifndef G16_DIAG_GELU
#define G16_DIAG_GELU 1
#endif
// diagnostics of the epilogue's cost (round 5, profiles/ab/gemm16_epilogue_pricing_r05.log):
// G16_DIAG_ST2=0 issues no second-output stores (GELU activation / SwiGLU dup);
// G16_DIAG_ST2_SMALL=1 folds the second output into its first 256 KB (L2-resident);
// G16_DEFER=1: the first phase after an epilogue waits only for the pieces issued before that
// epilogue's stores (vmcnt(4 + stores)).  Measured and removed: odd workgroups starting half an
// item late (stagger), the bias loads moved into the last k-tile (spills).
#ifndef G16_DIAG_ST2
#define G16_DIAG_ST2 1
#endif
#ifndef G16_DIAG_ST2_SMALL
#define G16_DIAG_ST2_SMALL 0
#endif
#ifndef G16_DEFER
#define G16_DEFER 0
#endif
// G16_EPI_SYNC: both groups' epilogues between the same pair of barriers (see the item loop)
#ifndef G16_EPI_SYNC
#define G16_EPI_SYNC 1
#endif

// The epilogue of one work item (registers only, no LDS).
template <int EPI>
ORION_DEVICE constexpr bool g16_has_bias() { return EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_GELU_BWD; }

// the bias of the wave's four column groups (8 consecutive n per lane after the swap)
template <int EPI>
ORION_DEVICE void g16_load_bias(const GemmArgs& g, const G16Item& it, int grp, int q, u32x4 (&bias4)[4]) {
  const int nw = it.n0 + grp * 128;
#pragma unroll
  for (int ap = 0; ap < 4; ++ap) {
    const int nb = nw + 16 * (2 * ap + (q & 1)) + 8 * (q >> 1), nc = nb < g.N ? nb : 0;
    if (EPI != EPI_GELU_BWD || g.bias) bias4[ap] = *reinterpret_cast<const u32x4*>(g.bias + nc);
    else bias4[ap] = u32x4{0u, 0u, 0u, 0u};
  }
}

// EPI_ROPE: rotate the wave's accumulators in place (before the bf16 rounding: one rounding
// instead of the GEMM's plus the separate rope pass's).  The wave's 128 columns are aligned to
// 128, so they hold one head of RD = 128, and column n + 64 sits in accumulator tile a + 4 of
// the same lane and register: acc[a][b][r] is column nw + 16 a + 4 q + r of row mw + 16 b +
// i16.  The tables are read as 16-byte rows (4 d).  (RD = 64 -- two heads per wave, partner
// tile a + 2 -- is the same code, but instantiating both forms in one kernel spills.)
template <int RD>
ORION_DEVICE void g16_rope(const GemmArgs& g, f32x4 (&acc)[8][4], int mw, int q, int i16) {
  constexpr int HB = RD / 32;  // accumulator tiles per half head
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int mc = min(mw + 16 * b + i16, g.M - 1);
    const float* cr = g.rcos + (long)(mc % g.rT + g.rpos0) * (RD / 2) + 4 * q;
    const float* sr = g.rsin + (long)(mc % g.rT + g.rpos0) * (RD / 2) + 4 * q;
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      if ((a / HB) & 1) continue;  // second half of a head: rotated with its partner
      const int d = (a % HB) * 16;
      const f32x4 c = *reinterpret_cast<const f32x4*>(cr + d);
      const f32x4 sn = *reinterpret_cast<const f32x4*>(sr + d);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x1 = acc[a][b][r], x2 = acc[a + HB][b][r];
        acc[a][b][r] = x1 * c[r] - x2 * sn[r];
        acc[a + HB][b][r] = x2 * c[r] + x1 * sn[r];
      }
    }
    // one row's table reads in flight at a time (hoisting all 32 spills)
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int EPI>
ORION_DEVICE void g16_epilogue(const GemmArgs& g, f32x4 (&acc)[8][4], const G16Item& it, int wm, int grp,
                               int q, int i16, u32x4 (&bias4)[4]) {
  const int m0 = it.m0, kc = it.kc, rows_m = it.rows_m;
  const int mw = m0 + wm * 64;           // this wave's 64-row block
  const int nw = it.n0 + grp * 128;      // this wave's 128 columns
  if constexpr (EPI == EPI_ROPE) {
    if (nw < g.rcols) {  // wave-uniform: the q | k heads
      g16_rope<128>(g, acc, mw, q, i16);  // rD == 128 (orion_gemm_rope checks)
    }
  }
  if constexpr (EPI == EPI_WGRAD) {
    // fp32 partial tile into slab kc, or the final gradient (fp32 arena or bf16, scaled,
    // optionally accumulated): register quadruple = 4 consecutive n of row m
    float* slab = g.ksplit > 1 ? g.slabs + (long)kc * g.M * g.N : nullptr;
    const float wsc = (g.ksplit == 1 && g.scale) ? *g.scale : 1.f;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int m = mw + 16 * b + i16;
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const int n = nw + 16 * a + 4 * q;
        if (m < g.M && n < g.N) {
          const long o = (long)m * g.N + n;
          f32x4 v = acc[a][b];
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
    return;
  }
  // output resources based at row m0 (32-bit offsets cover one 256-row band)
  const __amdgpu_buffer_rsrc_t ro =
      make_rsrc(g.out + (long)m0 * g.ldo, (unsigned)(((long)(rows_m - 1) * g.ldo + g.N) * 2));
  [[maybe_unused]] __amdgpu_buffer_rsrc_t ro2 = ro;
  // a second output: GELU activation, SwiGLU' dup, SwiGLU h (written by the up half, ap 2 / 3)
  constexpr bool TWO = EPI == EPI_BIAS_GELU || EPI == EPI_SWIGLU_BWD || EPI == EPI_SWIGLU;
  if constexpr (TWO)
    ro2 = make_rsrc(g.out2 + (long)m0 * g.ldo2,
                    (unsigned)(((long)(rows_m - 1) * g.ldo2 + (EPI == EPI_SWIGLU ? g.N >> 1 : g.N)) * 2));
  // EPI_SWIGLU: tile column c of the wave -> output column (gate f, or up F + f) and h column f
  auto ocol = [&](int c) {
    if constexpr (EPI != EPI_SWIGLU) return c;
    const int off = c - nw;
    return (nw >> 1) + off + (off >= 64 ? (g.N >> 1) - 64 : 0);
  };
  auto ocol2 = [&](int c) { return EPI == EPI_SWIGLU ? (nw >> 1) + c - nw - 64 : c; };
  constexpr bool CS = EPI == EPI_GELU_BWD;
  // bf16 pair word -> two floats (low half first)
  auto unpack2 = [](unsigned w) { return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xFFFF0000u)}; };
  // Every epilogue operand (bias, GELU' pre-activations) is loaded up front, before the first
  // store: a load after a store is kept behind it (they may alias) and then waited with
  // vmcnt(0), which on CDNA4 also waits for the stores -- the GELU' epilogue ran as 17
  // serial HBM round trips per wave.  The fragment registers of the main loop are dead here.
  auto ncol = [&](int ap) { return nw + 16 * (2 * ap + (q & 1)) + 8 * (q >> 1); };
  if constexpr (g16_has_bias<EPI>()) g16_load_bias<EPI>(g, it, grp, q, bias4);
  // GELU' / SwiGLU' operands (the pre-activation, or the gate and up halves of the packed
  // gate_up projection) stream in one column group (ap) ahead of their use: the loads of group
  // ap + 1 are issued before the stores of group ap, so waiting for them never waits for those
  // stores, and only two groups' operands are live (32 / 64 VGPRs instead of 64 / 128)
  constexpr bool PRE = EPI == EPI_GELU_BWD || EPI == EPI_SWIGLU_BWD;
  [[maybe_unused]] __amdgpu_buffer_rsrc_t rp;
  if constexpr (PRE)
    rp = make_rsrc(g.pre + (long)m0 * g.ldp,
                   (unsigned)(((long)(rows_m - 1) * g.ldp + (EPI == EPI_SWIGLU_BWD ? 2 : 1) * g.N) * 2));
  auto load_pre = [&](int ap, u32x4 (&pa)[4], u32x4 (&pb)[4]) {
    const int nb = ncol(ap), nc = nb < g.N ? nb : 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int mc = min(mw + 16 * b + i16, g.M - 1);
      const unsigned o = (unsigned)(((long)(mc - m0) * g.ldp + nc) * 2);
      pa[b] = __builtin_amdgcn_raw_buffer_load_b128(rp, o, 0, 0);
      if constexpr (EPI == EPI_SWIGLU_BWD)  // up half: F columns further
        pb[b] = __builtin_amdgcn_raw_buffer_load_b128(rp, o + (unsigned)g.N * 2, 0, 0);
    }
  };
  [[maybe_unused]] u32x4 preA[4], preB[4], upA[4], upB[4];
  if constexpr (PRE) load_pre(0, preA, upA);
  [[maybe_unused]] u32x4 parkA[4], parkB[4];  // G16_WIDE_ST: packed results of the even pair
  // LM head: the lane's four rows' targets / scales, the exp reference, row-sum accumulators
  constexpr float L2E = 1.4426950408889634f;
  [[maybe_unused]] int tg[4];
  [[maybe_unused]] float rsb[4], rsum[4];
  [[maybe_unused]] f32x2 cl2;
  if constexpr (EPI == EPI_EXP || EPI == EPI_ROWSCALE) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int mc = min(mw + 16 * b + i16, g.M - 1);
      if constexpr (EPI == EPI_EXP) {
        const long t = g.tgt[mc];
        tg[b] = (t >= 0 && t < g.N) ? (int)t : -1;
        rsum[b] = 0.f;
      } else {
        rsb[b] = g.rs[mc];
      }
    }
    if constexpr (EPI == EPI_EXP) cl2 = splat2(-*g.cref * L2E);
  }

  // the value arithmetic runs on pairs of adjacent columns (v_pk_*_f32: no MFMA issues beside
  // the epilogue) and every pair is packed to bf16 by one v_cvt_pk_bf16_f32
#pragma unroll
  for (int ap = 0; ap < 4; ++ap) {
    // after the swap: lane (q, i16) holds n = nb .. nb + 7 of row m (fp32)
    const int nb = ncol(ap);
    const bool nok = nb < g.N;
    if constexpr (PRE) {
      if (ap + 1 < 4) {
        if (ap & 1) load_pre(ap + 1, preA, upA);
        else load_pre(ap + 1, preB, upB);
      }
    }

    [[maybe_unused]] f32x2 bias[4];
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_GELU_BWD) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bias[e] = unpack2(bias4[ap][e]);
    }
    [[maybe_unused]] f32x2 cs[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int m = mw + 16 * b + i16;
      [[maybe_unused]] u32x4 p4, u4;
      if constexpr (PRE) {
        p4 = (ap & 1) ? preB[b] : preA[b];
        u4 = (ap & 1) ? upB[b] : upA[b];
      }
      f32x2 v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * ap][b][r]),
                                                         __float_as_uint(acc[2 * ap + 1][b][r]), false, false);
        v[r >> 1][r & 1] = __uint_as_float(sw[0]);
        v[2 + (r >> 1)][r & 1] = __uint_as_float(sw[1]);
      }
      if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bias[e];
      }
      if constexpr (EPI == EPI_GELU_BWD) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (g.deriv) v[e] *= unpack2(p4[e]);  // pre holds GELU'(a) (bias already inside)
          else v[e] *= G16_DIAG_GELU ? gelu_grad_x2(unpack2(p4[e]) + bias[e]) : unpack2(p4[e]) + bias[e];
        }
      }
      if constexpr (EPI == EPI_EXP) {
        // the target's logit (fp32, before the exp) for the loss; exp(acc - cref) and its row sum
        const int d = tg[b] - nb;
        if (d >= 0 && d < 8 && m < g.M) {
          float tl = 0.f;  // v[d >> 1][d & 1] without a runtime register index (scratch)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if ((d >> 1) == e) tl = (d & 1) ? v[e].y : v[e].x;
          g.tlog[m] = tl;
        }
        f32x2 se = splat2(0.f);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const f32x2 z = fma2(v[e], splat2(L2E), cl2);
          v[e] = f32x2{__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)};
          se += v[e];
        }
        if (nok) rsum[b] += se.x + se.y;
      }
      if constexpr (EPI == EPI_ROWSCALE) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] *= splat2(rsb[b]);
      }
      [[maybe_unused]] f32x2 du[4];
      if constexpr (EPI == EPI_SWIGLU) {
        // up half: h = silu(gate) up, the gate of the same columns from tiles 2 (ap - 2) (+ 1)
        if (ap >= 2) {
          f32x2 vg[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * ap - 4][b][r]),
                                                             __float_as_uint(acc[2 * ap - 3][b][r]), false, false);
            vg[r >> 1][r & 1] = __uint_as_float(sw[0]);
            vg[2 + (r >> 1)][r & 1] = __uint_as_float(sw[1]);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) du[e] = vg[e] * sigmoid2(vg[e]) * v[e];
        }
      }
      if constexpr (EPI == EPI_SWIGLU_BWD) {
        // v = dh; dgate = dh u silu'(g), dup = dh silu(g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const f32x2 gg = unpack2(p4[e]), uu = unpack2(u4[e]);
          const f32x2 sg = sigmoid2(gg);
          du[e] = v[e] * gg * sg;
          v[e] = v[e] * uu * fma2(gg * sg, splat2(1.f) - sg, sg);
        }
      }
      u32x4 pk, pk2;
      if (EPI == EPI_BIAS_GELU && G16_DIAG_GELU && g.deriv) {  // (GELU'(a), gelu(a))
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          f32x2 ge, de;
          gelu_and_grad_x2(v[e], ge, de);
          pk[e] = pack2_bf16(de);
          pk2[e] = pack2_bf16(ge);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) pk[e] = pack2_bf16(v[e]);
        if constexpr (TWO) {
          if (EPI != EPI_SWIGLU || ap >= 2) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              if constexpr (EPI == EPI_BIAS_GELU) pk2[e] = pack2_bf16(G16_DIAG_GELU ? gelu_x2(v[e]) : v[e] * v[e]);
              else pk2[e] = pack2_bf16(du[e]);
            }
          }
        }
      }
      // bias + GELU: the pre-activation is read again only by the backward -- streamed past
      // the caches (G16_PRE_NT)
      constexpr int AUX1 = (EPI == EPI_BIAS_GELU && G16_PRE_NT) ? 2 : G16_ST_AUX;
      if constexpr (G16_WIDE_ST) {
        // even column pair: park; odd pair: exchange lane bit 3 (row i16 & 8) with the pair
        // index, so that store 0 covers rows 0-7 and store 1 rows 8-15 of this 16-row group,
        // each over both pairs' 32 + 32 columns (8 rows x 128 B)
        if ((ap & 1) == 0) {
          parkA[b] = pk;
          if constexpr (TWO) {
            if (EPI != EPI_SWIGLU || ap >= 2) parkB[b] = pk2;
          }
        } else {
          const int hi = (i16 >> 3) & 1;
          auto xchg = [&](const u32x4& a, const u32x4& bb, u32x4& n0, u32x4& n1) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              // row_ror:8 (dpp_ctrl 0x128) reads lane i16 ^ 8; banks 2-3 are lanes 8-15 of a row
              n0[e] = (unsigned)__builtin_amdgcn_update_dpp((int)a[e], (int)bb[e], 0x128, 0xF, 0xC, false);
              n1[e] = (unsigned)__builtin_amdgcn_update_dpp((int)bb[e], (int)a[e], 0x128, 0xF, 0x3, false);
            }
          };
          u32x4 n0, n1;
          xchg(parkA[b], pk, n0, n1);
          // after the exchange lane (q, i16) holds column pair ap - 1 + hi of rows
          // 16 b + (i16 & 7) (n0) and 16 b + 8 + (i16 & 7) (n1)
          const int ncx = nw + 16 * (2 * (ap - 1 + hi) + (q & 1)) + 8 * (q >> 1);
          const int mr0 = mw + 16 * b + (i16 & 7), mr1 = mr0 + 8;
          const bool nx = ncx < g.N;
          const int oc = ocol(ncx);
          const unsigned o0 = (mr0 < g.M && nx) ? (unsigned)(((long)(mr0 - m0) * g.ldo + oc) * 2) : 0xFFFFFFF0u;
          const unsigned o1 = (mr1 < g.M && nx) ? (unsigned)(((long)(mr1 - m0) * g.ldo + oc) * 2) : 0xFFFFFFF0u;
          __builtin_amdgcn_raw_buffer_store_b128(n0, ro, o0, 0, AUX1);
          __builtin_amdgcn_raw_buffer_store_b128(n1, ro, o1, 0, AUX1);
          if (TWO && G16_DIAG_ST2 && (EPI != EPI_SWIGLU || ap == 3)) {
            xchg(parkB[b], pk2, n0, n1);
            const int oc2 = ocol2(ncx);
            unsigned p0 = (mr0 < g.M && nx) ? (unsigned)(((long)(mr0 - m0) * g.ldo2 + oc2) * 2) : 0xFFFFFFF0u;
            unsigned p1 = (mr1 < g.M && nx) ? (unsigned)(((long)(mr1 - m0) * g.ldo2 + oc2) * 2) : 0xFFFFFFF0u;
#if G16_DIAG_ST2_SMALL  // diagnostic: the second output folded into its first 256 KB (L2-resident)
            p0 &= 0x3FFF0u;
            p1 &= 0x3FFF0u;
#endif
            __builtin_amdgcn_raw_buffer_store_b128(n0, ro2, p0, 0, G16_ST2_AUX);
            __builtin_amdgcn_raw_buffer_store_b128(n1, ro2, p1, 0, G16_ST2_AUX);
          }
        }
      } else {
        const bool ok = m < g.M && nok;
        const unsigned off = ok ? (unsigned)(((long)(m - m0) * g.ldo + ocol(nb)) * 2) : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_buffer_store_b128(pk, ro, off, 0, AUX1);
        if (TWO && (EPI != EPI_SWIGLU || ap >= 2)) {
          const unsigned off2 = ok ? (unsigned)(((long)(m - m0) * g.ldo2 + ocol2(nb)) * 2) : 0xFFFFFFF0u;
          __builtin_amdgcn_raw_buffer_store_b128(pk2, ro2, off2, 0, G16_ST2_AUX);
        }
      }
      if constexpr (CS) {
        const f32x2 keep = splat2(m < g.M ? 1.f : 0.f);  // rows past M repeat row M - 1
#pragma unroll
        for (int e = 0; e < 4; ++e) cs[e] = b ? fma2(keep, v[e], cs[e]) : keep * v[e];
      }
    }
    if constexpr (CS) {
      if (g.colsum) {
        float c8[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          c8[2 * e] = cs[e].x;
          c8[2 * e + 1] = cs[e].y;
        }
        // sum over the 16 lanes of each row group (same n, m = i16): three halving exchange
        // steps (at offset o a lane keeps the half of its live values selected by lane bit o
        // and adds its partner's copy of it), then one full add with lane ^ 1; lane i16 ends
        // with value index (i16 >> 1) & 7
        auto step = [&](auto Oc) {
          constexpr int o = decltype(Oc)::value, half = o / 2;
          const bool up = (i16 & o) != 0;
#pragma unroll
          for (int k = 0; k < half; ++k) {
            const float send = up ? c8[k] : c8[half + k];
            const float keep = up ? c8[half + k] : c8[k];
            c8[k] = keep + __shfl_xor(send, o);
          }
        };
        step(std::integral_constant<int, 8>());
        step(std::integral_constant<int, 4>());
        step(std::integral_constant<int, 2>());
        const float tot = c8[0] + __shfl_xor(c8[0], 1);
        const int n = nb + ((i16 >> 1) & 7);
        if (!(i16 & 1) && mw < g.M && n < g.N) g.colsum[(long)(mw / 64) * g.N + n] = tot;
      }
    }
  }
  if constexpr (EPI == EPI_EXP) {
    // the four q lanes of a row hold its 128 columns: fold them, one partial per (row, wave)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      float r = rsum[b];
      r += __shfl_xor(r, 16);
      r += __shfl_xor(r, 32);
      const int m = mw + 16 * b + i16;
      // a wave whose 128 columns all lie past N (the last tile's second group when N % 256 <=
      // 128, e.g. GPT-2's 50,304) has no partial: its index would be the next row's part 0
      if (q == 0 && m < g.M && nw < g.N) g.rowpart[(long)m * g.npart + nw / 128] = r;
    }
  }
}

// STAMPS (diagnostic instantiation: ORION_GEMM_DIAG=4 with a stamp buffer, EPI_STORE / BIAS /
// BIAS_GELU, one item per workgroup or (flags & 128) the persistent walk): every wave of every workgroup records s_memtime at 16 points --
// kernel start, prologue landed, the 6 slot boundaries of both phases of the middle k-tile
// (READ start, reads+DMA issued, vmcnt retired, MMA slot entered, fragments landed, MFMAs
// issued), main loop done, epilogue issued -- plus where it ran (HW_ID / XCC_ID) into g.slabs
// as u64 [workgroup][wave][20] (scripts/gemm16_stamps.py, scripts/gemm16_timeline.py).
template <bool XKM, bool WKM, int EPI, bool STAMPS = false>
__global__ __launch_bounds__(512, 1) void gemm16_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wv >> 2, wm = wv & 3;
  const int q = lane >> 4, i16 = lane & 15;
  [[maybe_unused]] unsigned long stp[20] = {};
  if constexpr (STAMPS) stp[0] = __builtin_amdgcn_s_memtime();

  // this workgroup's items: the work ids of XCD group b % 8 are one contiguous range of the
  // grouped order (bijective split of `work` over 8), walked with stride = the number of
  // blocks of that group; with one block per item (grid = work) each block gets one item
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid & 7, lcl = bid >> 3;
  const int tiles_m = (g.M + 255) >> 8, work = tiles_m * g.tiles_n * g.ksplit;
  const int wq = work >> 3, wr = work & 7;
  const int r0 = xcd < wr ? xcd * (wq + 1) : wr * (wq + 1) + (xcd - wr) * wq;
  const int rlen = wq + (xcd < wr ? 1 : 0);
  const int stride = (nwg >> 3) + (xcd < (nwg & 7) ? 1 : 0);
  const int nitems = lcl < rlen ? (rlen - lcl + stride - 1) / stride : 0;
  if (nitems == 0) return;
  auto item_id = [&](int j) { return r0 + lcl + j * stride; };
  auto decode = [&](int j) { return g16_decode(g, item_id(j)); };

  const unsigned xstep = XKM ? (unsigned)(G_BK * g.ldx * 2) : G_BK * 2;
  const unsigned wstep = WKM ? (unsigned)(G_BK * g.ldw * 2) : G_BK * 2;

  // LDS-DMA of piece p (0 A, 1 B, 2 C, 3 D): this wave's blocks e = 0, 1 (one block = 8 image
  // rows x 128 bytes = one wave instruction: lane -> row lane / 8, 16-byte slot lane % 8).
  // LDS destinations (ld) are item-independent; the source offsets (vo) and the buffer
  // resources (based at the item's tile rows and k chunk, so only the tile's own extent has
  // to fit the 32-bit offsets: a 6.6 GB logits operand is fine) are set per item, separately
  // for the X stream and the W stream, which run ahead of the MFMAs by different amounts.
  unsigned vo[4][2];
  int ld[4][2];
  __amdgpu_buffer_rsrc_t rx, rw;
  const int lr = lane >> 3, slot = lane & 7;
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int b = 2 * wm + e;  // 0..7
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      if constexpr (XKM) ld[1 + jj][e] = (2 * jj + grp) * 4096 + 8 * b * 64;
      else ld[1 + jj][e] = ((2 * grp + (b >> 2)) * 64 + jj * 32 + (b & 3) * 8) * 64;
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int p = hh ? 3 : 0;
      if constexpr (WKM) ld[p][e] = (2 * grp + hh) * 4096 + 8 * b * 64;
      else ld[p][e] = (grp * 128 + hh * 64 + b * 8) * 64;
    }
  }
  auto setup_x = [&](const G16Item& it) {
    if constexpr (XKM)
      rx = make_rsrc(g.X + (long)it.k0 * g.ldx + it.m0, (unsigned)(((long)(it.kr - 1) * g.ldx + it.rows_m) * 2));
    else
      rx = make_rsrc(g.X + (long)it.m0 * g.ldx + it.k0, (unsigned)(((long)(it.rows_m - 1) * g.ldx + it.kr) * 2));
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int b = 2 * wm + e;
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {  // X pieces B (jj 0), C (jj 1)
        if constexpr (XKM) {  // [64 k][64 m] image of wave row block wmp
          const int wmp = 2 * jj + grp, k = 8 * b + lr;
          const int m = it.m0 + wmp * 64 + 8 * (slot ^ (km_swz(k) << 1));
          vo[1 + jj][e] = (unsigned)(((long)k * g.ldx + min(m, g.M - 8) - it.m0) * 2);
        } else {  // [256 m][64 k]: rows wm' 64 + 32 jj + [0, 32)
          const int row0 = (2 * grp + (b >> 2)) * 64 + jj * 32 + (b & 3) * 8, row = row0 + lr;
          const int ch = slot ^ nt_swz(row);
          vo[1 + jj][e] = (unsigned)(((long)(min(it.m0 + row, g.M - 1) - it.m0) * g.ldx + 8 * ch) * 2);
        }
      }
    }
  };
  auto setup_w = [&](const G16Item& it) {
    if constexpr (WKM)
      rw = make_rsrc(g.W + (long)it.k0 * g.ldw + it.n0, (unsigned)(((long)(it.kr - 1) * g.ldw + it.rows_n) * 2));
    else if constexpr (EPI == EPI_SWIGLU)  // gate and up rows F apart: the whole W (orion_gemm_swiglu checks)
      rw = make_rsrc(g.W + it.k0, (unsigned)(((long)(g.N - 1) * g.ldw + it.kr) * 2));
    else
      rw = make_rsrc(g.W + (long)it.n0 * g.ldw + it.k0, (unsigned)(((long)(it.rows_n - 1) * g.ldw + it.kr) * 2));
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int b = 2 * wm + e;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {  // W pieces A (n-half 0), D (n-half 1) of this group
        const int p = hh ? 3 : 0;
        if constexpr (WKM) {  // [64 k][64 n] image (grp, hh)
          const int k = 8 * b + lr;
          const int col = it.n0 + grp * 128 + hh * 64 + 8 * (slot ^ (km_swz(k) << 1));
          vo[p][e] = (unsigned)(((long)k * g.ldw + min(col, g.N - 8) - it.n0) * 2);
        } else {  // [256 n][64 k]: rows grp 128 + hh 64 + [0, 64)
          const int row0 = grp * 128 + hh * 64 + b * 8, row = row0 + lr;
          const int ch = slot ^ nt_swz(row);
          if constexpr (EPI == EPI_SWIGLU) {  // image row -> gate row f (hh 0) / up row F + f (hh 1)
            const int f = ((it.n0 + grp * 128) >> 1) + b * 8 + lr;
            vo[p][e] = (unsigned)(((long)(f + hh * (g.N >> 1)) * g.ldw + 8 * ch) * 2);
          } else {
            vo[p][e] = (unsigned)(((long)(min(it.n0 + row, g.N - 1) - it.n0) * g.ldw + 8 * ch) * 2);
          }
        }
      }
    }
  };
  auto ximg = [&](int s) -> bf16_t* { return smem + G_X0 + (s % 3) * G_IMG; };
  auto wimg = [&](int s) -> bf16_t* { return smem + G_W0 + (s & 1) * G_IMG; };

  // the two issue streams: item index, k-tile within it, global k-tile counter (LDS buffer)
  int jx = 0, tx = 0, sx = 0, jw = 0, tw = 0, sw = 0;
  int nkx, nkw;
  {
    const G16Item it = decode(0);
    setup_x(it);
    setup_w(it);
    nkx = nkw = it.nk;
  }
  auto issue_x = [&](int jj) {  // piece B (jj 0) / C (jj 1) of the X stream's k-tile
    ORION_DASSERT(jx < nitems && tx < nkx);
    bf16_t* base = ximg(sx);
#pragma unroll
    for (int e = 0; e < 2; ++e) blds16(rx, vo[1 + jj][e], (unsigned)tx * xstep, base + ld[1 + jj][e]);
  };
  auto issue_w = [&](int hh) {  // piece A (hh 0) / D (hh 1) of the W stream's k-tile
    ORION_DASSERT(jw < nitems && tw < nkw);
    bf16_t* base = wimg(sw);
    const int p = hh ? 3 : 0;
#pragma unroll
    for (int e = 0; e < 2; ++e) blds16(rw, vo[p][e], (unsigned)tw * wstep, base + ld[p][e]);
  };
  // A stream that has issued its last k-tile stays on it: the DMA of the final one or two
  // steps re-loads that tile into a buffer no phase reads any more, so every phase issues the
  // same pieces and waits the same count (no branches in the steady state); the kernel drains
  // them (vmcnt(0)) before it ends.
  auto advance_x = [&]() {
    ++sx;
    if (tx + 1 < nkx) {
      ++tx;
    } else if (jx + 1 < nitems) {
      ++jx;
      tx = 0;
      const G16Item it = decode(jx);
      setup_x(it);
      nkx = it.nk;
    }
  };
  auto advance_w = [&]() {
    ++sw;
    if (tw + 1 < nkw) {
      ++tw;
    } else if (jw + 1 < nitems) {
      ++jw;
      tw = 0;
      const G16Item it = decode(jw);
      setup_w(it);
      nkw = it.nk;
    }
  };

  // per-lane fragment offsets (bytes).  NT: row i16 of a 16-row tile, k chunk 4 s + q.
  // k-major: rows 8 q + (i16 >> 2) (+ 4 for the second read, + 32 for k-step 1), columns
  // 16 tile + 4 (i16 & 3) with the 32-byte segment (= tile) XOR the row swizzle.
  int nto[2], kmo[4];
#pragma unroll
  for (int s = 0; s < 2; ++s) nto[s] = i16 * 128 + (((4 * s + q) ^ nt_swz(i16)) << 4);
  {
    const int row0 = 8 * q + (i16 >> 2), h = km_swz(row0);
#pragma unroll
    for (int b = 0; b < 4; ++b) kmo[b] = row0 * 128 + ((b ^ h) << 5) + 8 * (i16 & 3);
  }
  const unsigned lds0 = lds_addr(smem, 0);

  f32x4 acc[8][4];
  // fragments: W [tile][k-step] (n-half 0 / 1), X [m-tile] of k-step 0 and of k-step 1
  bf16x8 W0[4][2], W1[4][2], X0[4], X1[4];

  // the wave's 4 m-tile fragments of k-step S of the k-tile in LDS buffer s
  auto read_x = [&](bf16x8 (&Xd)[4], int s, auto Sc) {
    constexpr int S = decltype(Sc)::value;
    const unsigned base = lds0 + (unsigned)(ximg(s) - smem) * 2 + wm * 8192;
    if constexpr (XKM) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const unsigned a = base + kmo[b];
        Xd[b] = cat8(rd_tr<4096 * S>(a), rd_tr<4096 * S + 512>(a));
      }
    } else {
      const unsigned a = base + nto[S];
      Xd[0] = rd_b128<0>(a);
      Xd[1] = rd_b128<2048>(a);
      Xd[2] = rd_b128<4096>(a);
      Xd[3] = rd_b128<6144>(a);
    }
  };
  // W fragments of n-half H of the k-tile in buffer s: 4 n-tiles x 2 k-steps
  auto read_w = [&](bf16x8 (&Wf)[4][2], int s, auto Hc) {
    constexpr int H = decltype(Hc)::value;
    if constexpr (WKM) {
      const unsigned base = lds0 + (unsigned)(wimg(s) - smem) * 2 + (2 * grp + H) * 8192;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const unsigned ad = base + kmo[a];
        Wf[a][0] = cat8(rd_tr<0>(ad), rd_tr<512>(ad));
        Wf[a][1] = cat8(rd_tr<4096>(ad), rd_tr<4608>(ad));
      }
    } else {
      const unsigned base = lds0 + (unsigned)(wimg(s) - smem) * 2 + grp * 16384 + H * 8192;
      const unsigned a0 = base + nto[0], a1 = base + nto[1];
      Wf[0][0] = rd_b128<0>(a0);
      Wf[0][1] = rd_b128<0>(a1);
      Wf[1][0] = rd_b128<2048>(a0);
      Wf[1][1] = rd_b128<2048>(a1);
      Wf[2][0] = rd_b128<4096>(a0);
      Wf[2][1] = rd_b128<4096>(a1);
      Wf[3][0] = rd_b128<6144>(a0);
      Wf[3][1] = rd_b128<6144>(a1);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  // stamped item: the only one (one workgroup per item) or, on the persistent walk (flags &
  // 128), the middle one; its successor's first k-tile stamps its wait / barrier exits
  [[maybe_unused]] const bool spers = STAMPS && (g.flags & 128);
  [[maybe_unused]] const int jsel = spers && nitems >= 3 ? nitems / 2 : 0;
  int tsel = -1, jcur = 0;
  auto stamp = [&](int t, int k) {
    if constexpr (STAMPS) {
      if (t == tsel && jcur == jsel) stp[k] = __builtin_amdgcn_s_memtime();
      if (spers && t == 0 && jcur == jsel + 1 && (k == 4 || k == 5 || k == 10 || k == 11))
        stp[16 + (k & 1) + (k >= 10 ? 2 : 0)] = __builtin_amdgcn_s_memtime();
    }
  };
  // one phase of global k-tile s (k-tile t of the current item): READ slot (fragments + the
  // streams' pieces, then vmcnt(<this phase's own loads>), so every older piece has landed
  // before the next phase), MMA slot (32 MFMAs)
  // stores a wave issues in every non-WGRAD epilogue (at least): G16_DEFER's wait count
  constexpr int NST = !G16_DIAG_ST2 ? 16 : (EPI == EPI_BIAS_GELU || EPI == EPI_SWIGLU_BWD) ? 32 : EPI == EPI_SWIGLU ? 24 : 16;
  [[maybe_unused]] u32x4 bias4[4];
  // tail: the item's last phase; its closing barrier is left to the caller (G16_EPI_SYNC)
  auto phase = [&](auto Hc, int s, int t, bool defer, bool tail) {
    constexpr int H = decltype(Hc)::value;
    stamp(t, 2 + 6 * H);
    if constexpr (H == 0) {
      read_w(W0, s, Hc);
      read_x(X0, s, I0());
      read_x(X1, s, I1());
    } else {
      read_w(W1, s, Hc);
    }
    issue_w(H);
    issue_x(H);
    stamp(t, 3 + 6 * H);
    if constexpr (H == 0 && G16_DEFER && EPI != EPI_WGRAD) {
      if (defer) wait_vm_exact<4 + NST>();
      else wait_vm_exact<4>();
    } else {
      wait_vm_exact<4>();
    }
    stamp(t, 4 + 6 * H);
    g_barrier();
    stamp(t, 5 + 6 * H);
    // every fragment an MFMA of this slot reads is retired (and pinned behind the wait)
    if constexpr (H == 0) {
      g_wait_lds(W0);
      asm volatile("" : "+v"(X0[0]), "+v"(X0[1]), "+v"(X0[2]), "+v"(X0[3]), "+v"(X1[0]),
                   "+v"(X1[1]), "+v"(X1[2]), "+v"(X1[3]));
    } else {
      g_wait_lds(W1);
    }
    __builtin_amdgcn_sched_barrier(0);
    stamp(t, 6 + 6 * H);
    bf16x8 (&Wf)[4][2] = H == 0 ? W0 : W1;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[4 * H + a][b] = mfma16(Wf[a][0], X0[b], acc[4 * H + a][b]);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[4 * H + a][b] = mfma16(Wf[a][1], X1[b], acc[4 * H + a][b]);
    __builtin_amdgcn_s_setprio(0);
    stamp(t, 7 + 6 * H);
    if (!tail) g_barrier();
  };

  // prologue: X k-tile 0 (B, C), W k-tile 0 (A, D), X k-tile 1 (B, C); phase (0, 0) needs the
  // first three pieces
  issue_x(0);
  issue_x(1);
  advance_x();
  issue_w(0);
  issue_w(1);
  advance_w();
  issue_x(0);
  issue_x(1);
  advance_x();
  wait_vm_exact<6>();
  if constexpr (STAMPS) stp[1] = __builtin_amdgcn_s_memtime();
  g_barrier();
  if (grp == 1) g_barrier();  // the stagger: group 1 runs one slot behind (kept across items)

  int s = 0;
  for (int j = 0; j < nitems; ++j) {
    const G16Item it = decode(j);
    if constexpr (STAMPS) {
      tsel = it.nk / 2;
      jcur = j;
    }
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = zero4();
    for (int t = 0; t < it.nk; ++t, ++s) {
      phase(I0(), s, t, t == 0 && j > 0, false);
      phase(I1(), s, t, false, t == it.nk - 1);
      advance_w();
      advance_x();
    }
    // The last phase's closing barrier.  Group 1 runs one slot behind group 0: with the
    // epilogue after that barrier in both groups (G16_EPI_SYNC 0) group 1 waits there through
    // group 0's whole epilogue and group 0 then waits through group 1's at its next one -- the
    // two epilogues run one after the other (scripts/gemm16_epi_stamps.py).  Group 1 runs its
    // epilogue before the barrier instead, so both groups' epilogues fall between the same
    // two barriers and run side by side.
    const bool epi_first = G16_EPI_SYNC && grp == 1;
    if (!epi_first) g_barrier();
    if constexpr (STAMPS) {
      if (j == jsel) stp[14] = __builtin_amdgcn_s_memtime();
    }
    g16_epilogue<EPI>(g, acc, it, wm, grp, q, i16, bias4);
    if constexpr (STAMPS) {
      if (spers && j == jsel) stp[15] = __builtin_amdgcn_s_memtime();
    }
    if (epi_first) g_barrier();
  }
  if (grp == 0) g_barrier();  // match group 1's barrier count
  wait_vm_exact<0>();         // the stream's last (dummy) LDS-DMA lands before the LDS is freed
  if constexpr (STAMPS) {
    // one item per workgroup: 15: epilogue issued; 16: where the wave ran (HW_ID: cu / sh /
    // se; XCC_ID); 17: its stores acknowledged (only with flags & 32, which waits for them:
    // the default leaves the wave to end right after issuing, as the real kernel does).
    // Persistent (flags & 128): 15 the stamped item's epilogue issued, 16-19 the next item's
    // first k-tile: phase 0 vmcnt retired, its barrier passed, phase 1 the same
    if (!spers) {
    stp[15] = __builtin_amdgcn_s_memtime();
    stp[16] = (unsigned long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
              ((unsigned long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
    stp[17] = 0;
    if (g.flags & 32) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stp[17] = __builtin_amdgcn_s_memtime();
    }
    }
    if (lane == 0) {
      unsigned long* dst = reinterpret_cast<unsigned long*>(g.slabs) + ((long)blockIdx.x * 8 + wv) * 20;
#pragma unroll
      for (int k = 0; k < 20; ++k) dst[k] = stp[k];
    }
  }
}

template <bool XKM, bool WKM, int EPI, bool STAMPS = false>
static int gemm16_launch(const GemmArgs& a, hipStream_t st) {
  if constexpr (!STAMPS && (EPI == EPI_STORE || EPI == EPI_BIAS || EPI == EPI_BIAS_GELU)) {
    if ((a.flags & 4) && a.slabs) return gemm16_launch<XKM, WKM, EPI, true>(a, st);
  }
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)gemm16_kernel<XKM, WKM, EPI, STAMPS>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, G_LDS) != hipSuccess)
      return -5;
    attr = true;
  }
  const long work = (long)((a.M + 255) / 256) * a.tiles_n * a.ksplit;
  if (work <= 0 || work > 0x7FFFFFFFL) return -1;
  // persistent walk (one workgroup per CU) unless a stamped diagnostic or flags & 64 asks for
  // one workgroup per item
  const bool one_per_item = (STAMPS && !(a.flags & 128)) || (a.flags & 64) || work <= 256;
  const unsigned grid = one_per_item ? (unsigned)work : 256u;
  gemm16_kernel<XKM, WKM, EPI, STAMPS><<<grid, 512, G_LDS, st>>>(a);
  return (int)hipGetLastError();
}

// 32-bit buffer offsets of one work item: a k-major operand spans its whole k chunk, an NT
// operand and the output one 256-row band
bool gemm16_ok(const GemmArgs& a, int wkm) {
  const long lim = 0xFFFFFF00L;
  const long band = 256L * (a.ldx > a.ldw ? a.ldx : a.ldw) * 2;
  const long ob = 256L * (a.ldo > a.ldo2 ? a.ldo : a.ldo2) * 2, pb = 256L * a.ldp * 2;
  const long wb = wkm ? (long)a.K * a.ldw * 2 : 0;
  return band < lim && ob < lim && pb < lim && wb < lim;
}

int gemm16_wgrad(const GemmArgs& a, int bt, hipStream_t st) {
  // bt: the second operand NT ([N2][tokens], the LM head's transposed scaled activations)
  return bt ? gemm16_launch<true, false, EPI_WGRAD>(a, st) : gemm16_launch<true, true, EPI_WGRAD>(a, st);
}

int gemm16(const GemmArgs& a0, int wkm, int epi, hipStream_t st) {
  GemmArgs a = a0;
  a.kchunk = a.K;
  a.ksplit = 1;
  switch (epi * 2 + (wkm ? 1 : 0)) {
    case EPI_STORE * 2 + 0: return gemm16_launch<false, false, EPI_STORE>(a, st);
    case EPI_STORE * 2 + 1: return gemm16_launch<false, true, EPI_STORE>(a, st);
    case EPI_BIAS * 2 + 0: return gemm16_launch<false, false, EPI_BIAS>(a, st);
    case EPI_BIAS_GELU * 2 + 0: return gemm16_launch<false, false, EPI_BIAS_GELU>(a, st);
    case EPI_GELU_BWD * 2 + 1: return gemm16_launch<false, true, EPI_GELU_BWD>(a, st);
    case EPI_SWIGLU_BWD * 2 + 1: return gemm16_launch<false, true, EPI_SWIGLU_BWD>(a, st);
    case EPI_EXP * 2 + 0: return gemm16_launch<false, false, EPI_EXP>(a, st);
    case EPI_ROWSCALE * 2 + 1: return gemm16_launch<false, true, EPI_ROWSCALE>(a, st);
    case EPI_ROPE * 2 + 0: return gemm16_launch<false, false, EPI_ROPE>(a, st);
    case EPI_SWIGLU * 2 + 0: return gemm16_launch<false, false, EPI_SWIGLU>(a, st);
    default: return -4;
  }
}

}  // namespace orion
