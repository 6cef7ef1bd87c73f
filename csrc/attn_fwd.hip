// Flash-attention forward, round-3 form (gfx950): the algorithm of attention.hip's
// attn_fwd_kernel (swapped S^T = K Q^T with the query on the lane, P straight from the
// accumulator into O^T += V^T P^T, online softmax in base 2 with a deferred rescale) with
// the per-tile instruction overhead taken out.  PMC of the older kernel at the GPT-2 shape
// (profiles/pmc_attn_r02m.txt): 16 vector instructions per MFMA and 25 % MFMA busy -- the
// kernel is bound by vector-instruction ISSUE, and half of those instructions were not
// softmax but bookkeeping:
//
//   * K / V staging by buffer loads: one per-thread 32-bit offset computed once, the tile
//     advance in the scalar soffset -- no 64-bit address multiply per load and tile (the
//     clamped path runs only for a last partial tile);
//   * the tile loop unrolled by the two LDS buffers, so every LDS read and write address is
//     a loop-invariant per-lane register plus an immediate;
//   * causal / length mask as one compare + select per score against a per-lane bound
//     (the per-element key arithmetic and exec-mask branches are gone), on diagonal tiles
//     only;
//   * row max and row sum as four independent chains (no 32-deep dependent chain);
//   * all K fragments of a tile read before its S MFMAs (ordered by sched_group_barrier),
//     so the MFMAs no longer wait on one LDS round trip each.
//
// One workgroup = 4 waves = 128 query rows (32 per wave), key tiles of 64 double-buffered
// in LDS, two workgroups per CU.  bf16 in / out, fp32 accumulation, O written as (B, T, H,
// D), lse in base 2.  attention.hip's older forward remains the 64-bit-addressed fallback
// (offsets past 2 GB; ORION_ATTN_FWD=v2 forces it for its test).
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "attn_params.h"
#include "mfma_lds.h"

#ifndef ATTN_FWD_QB64
#define ATTN_FWD_QB64 2  // query blocks per wave at D = 64 (A/B builds: -DATTN_FWD_QB64=1)
#endif

namespace orion {

// Plain fmaxf / + here: this file is built with -fno-honor-nans (no canonicalising
// v_max x, x per MFMA result, so max chains become v_max3) and -fno-slp-vectorize (adjacent
// f32 adds are not packed into v_pk_add_f32, which costs more than two plain adds beside
// MFMAs: MI355X_MICROARCH.md).  The same ops as inline asm miscomputed the diagonal tiles
// (the asm hides the VALU result hazards from the compiler's wait-state insertion).
ORION_DEVICE float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
ORION_DEVICE float addf(float a, float b) { return a + b; }

// the two 32-lane halves of a wave exchanged by one v_permlane32_swap: {x of lanes 0-31,
// x of lanes 32-63} in every lane (instead of __shfl_xor(x, 32)'s ds_bpermute round trip)
ORION_DEVICE float half_max(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}
ORION_DEVICE float half_sum(float x) {
  const unsigned u = __builtin_bit_cast(unsigned, x);
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}

ORION_DEVICE bf16x8 buf_load16(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// STAMPS (diagnostic instantiation, ORION_ATTN_FWD_DIAG=1, D = 64 causal): every wave sums
// s_memtime deltas of the five phases of a key tile (stage write + next load issue, K reads +
// S MFMA issue, softmax incl. the wait for S, V reads + PV issue, barrier) and writes them with
// its active-tile count, tile count and lifetime over p.o (scripts/attn_fwd_stamps.py).
template <int D, bool CAUSAL, int QB, bool STAMPS = false>
__global__ __launch_bounds__(256, 2) void attn_fwd3_kernel(AttnParams p) {
  // QB query blocks of 32 rows per wave (D = 64: 2, one 64-key tile's K / V fragments feed
  // both blocks' MFMAs and the two softmax chains interleave with each other's MFMAs)
  constexpr int BM = 128 * QB, BN = 64, NCH = D / 8, TILE = BN * D, NST = BN * NCH / 256, NDB = D / 32;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];  // [2 bufs][K|V][TILE]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h32 = lane >> 5, l32 = lane & 31;
  const int BH = p.B * p.Hq;
  const int nqt = (p.T + BM - 1) / BM;
  const int bh = blockIdx.x % BH;
  const int qt = nqt - 1 - (int)(blockIdx.x / BH);  // heaviest (causal) tiles launch first
  const int b = bh / p.Hq, hq = bh % p.Hq, hk = hq / (p.Hq / p.Hkv);
  const int q0 = qt * BM, qw0 = q0 + wv * 32 * QB;
  const int off = p.Tk - p.T;  // causal: key <= query + off
  const float c = p.scale_log2;

  const bf16_t* Qb = p.q + b * p.q_sb + hq * p.q_sh;
  const bf16_t* Kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* Vb = p.v + b * p.v_sb + hk * p.v_sh;

  bf16x8 qf[QB][D / 16];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const int qr = min(qw0 + qb * 32 + l32, p.T - 1);
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks)
      qf[qb][ks] = *reinterpret_cast<const bf16x8*>(Qb + (long)qr * p.q_st + ks * 16 + 8 * h32);
  }
  const int kend = CAUSAL ? min(p.Tk, q0 + BM + off) : p.Tk;
  const int ntiles = (kend + BN - 1) / BN;

  // staging: thread chunk i covers (row, ch) = ((tid + 256 i) / NCH, (tid + 256 i) % NCH)
  const unsigned kst_b = (unsigned)p.k_st * 2, vst_b = (unsigned)p.v_st * 2;  // bytes per key row
  const __amdgpu_buffer_rsrc_t rk = make_rsrc(Kb, (unsigned)((long)(p.Tk - 1) * p.k_st + D) * 2);
  const __amdgpu_buffer_rsrc_t rv = make_rsrc(Vb, (unsigned)((long)(p.Tk - 1) * p.v_st + D) * 2);
  unsigned vk[NST], vv[NST];
  int lo[NST];
#pragma unroll
  for (int i = 0; i < NST; ++i) {
    const int cidx = tid + i * 256, row = cidx / NCH, ch = cidx % NCH;
    vk[i] = row * kst_b + ch * 16;
    vv[i] = row * vst_b + ch * 16;
    lo[i] = loff<D>(row, ch * 8);
  }
  bf16x8 kst[NST], vst[NST];
  auto gload = [&](int t) {
    if (t * BN + BN <= p.Tk) {
      const unsigned sk = (unsigned)(t * BN) * kst_b, sv = (unsigned)(t * BN) * vst_b;
#pragma unroll
      for (int i = 0; i < NST; ++i) {
        kst[i] = buf_load16(rk, vk[i], sk);
        vst[i] = buf_load16(rv, vv[i], sv);
      }
    } else {  // last partial tile: rows past Tk re-read the last key (masked below)
#pragma unroll
      for (int i = 0; i < NST; ++i) {
        const int cidx = tid + i * 256, row = cidx / NCH, ch = cidx % NCH;
        const unsigned key = (unsigned)min(t * BN + row, p.Tk - 1);
        kst[i] = buf_load16(rk, key * kst_b + ch * 16, 0);
        vst[i] = buf_load16(rv, key * vst_b + ch * 16, 0);
      }
    }
  };
  auto swrite = [&](auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    bf16_t* Ks = smem + buf * 2 * TILE;
#pragma unroll
    for (int i = 0; i < NST; ++i) {
      *reinterpret_cast<bf16x8*>(Ks + lo[i]) = kst[i];
      *reinterpret_cast<bf16x8*>(Ks + TILE + lo[i]) = vst[i];
    }
  };

  // per-lane LDS fragment offsets (the same in both buffers)
  int ko[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) ko[ks] = loff<D>(l32, ks * 16 + 8 * h32);

  f32x16 oacc[QB][NDB];
  float m[QB], lsum[QB];
#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
#pragma unroll
    for (int db = 0; db < NDB; ++db) oacc[qb][db] = zero16();
    m[qb] = -1e30f;
    lsum[qb] = 0.f;
  }

  unsigned long long st_acc[5] = {0, 0, 0, 0, 0}, st_prev = 0, st_begin = 0;
  int st_n = 0;
  auto stamp = [&](int k) {
    if constexpr (STAMPS) {
      __builtin_amdgcn_sched_barrier(0);
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      if (k >= 0) st_acc[k] += t - st_prev;
      st_prev = t;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto tile = [&](auto bufc, int t) {
    constexpr int buf = decltype(bufc)::value;
    stamp(-1);
    if (t + 1 < ntiles) swrite(std::integral_constant<int, buf ^ 1>{});
    if (t + 2 < ntiles) gload(t + 2);
    stamp(0);
    const int k0 = t * BN;
    const bf16_t* Ks = smem + buf * 2 * TILE;
    const bf16_t* Vs = Ks + TILE;
    const bool active = !CAUSAL || (k0 <= qw0 + 32 * QB - 1 + off);
    if (active) {
      // K fragment reads issue before the S MFMAs that use them: all 8 at D = 64; one key
      // block (8 of 16) at a time at D = 128, where 64 fragment registers would spill
      constexpr int KBR = D == 64 ? 2 : 1;  // key blocks per read group
      f32x16 s[QB][2];
      mfma_prio(true);
#pragma unroll
      for (int kg = 0; kg < 2; kg += KBR) {
        bf16x8 kfr[KBR][D / 16];
#pragma unroll
        for (int kb = 0; kb < KBR; ++kb)
#pragma unroll
          for (int ks = 0; ks < D / 16; ++ks) kfr[kb][ks] = lds_b128(Ks + (kg + kb) * 32 * D, ko[ks]);
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
          for (int kb = 0; kb < KBR; ++kb) {
            s[qb][kg + kb] = zero16();
#pragma unroll
            for (int ks = 0; ks < D / 16; ++ks) s[qb][kg + kb] = mfma32(kfr[kb][ks], qf[qb][ks], s[qb][kg + kb]);
          }
        __builtin_amdgcn_sched_group_barrier(0x100, KBR * (D / 16), 0);
        __builtin_amdgcn_sched_group_barrier(0x008, QB * KBR * (D / 16), 0);
      }
      mfma_prio(false);
      stamp(1);
      ++st_n;
      bf16x8 pf[QB][4];
      float alpha[QB];
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        const int qwb = qw0 + qb * 32;
        const bool need_mask = (CAUSAL && (k0 + BN - 1 > qwb + off)) || (k0 + BN > p.Tk);
        if (need_mask) {
          // key k0 + kb*32 + rowoff(r) + 4*h32 is visible iff rowoff(r) <= lim
          // as min(s, (lim - rowoff + 0.5) * 1e35): >= 5e34 where visible (s unchanged), <= -5e34
          // where not (exp2 of it is 0, and it stays below the running max's -1e30 start) --
          // one fma + one min per score instead of a compare, the VCC hazard wait and a select
          const int vis = CAUSAL ? min(qwb + l32 + off, p.Tk - 1) : p.Tk - 1;
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) {
            if constexpr (CAUSAL && D == 64 && QB == 2) {  // elsewhere the constants cost registers (spills)
              const float fl = (float)(vis - (k0 + kb * 32 + 4 * h32));
#pragma unroll
              for (int r = 0; r < 16; ++r)
                s[qb][kb][r] = fminf(s[qb][kb][r], fmaf(fl, 1e35f, (0.5f - (float)((r & 3) + 8 * (r >> 2))) * 1e35f));
            } else {
              const int lim = vis - (k0 + kb * 32 + 4 * h32);
#pragma unroll
              for (int r = 0; r < 16; ++r)
                s[qb][kb][r] = ((r & 3) + 8 * (r >> 2) > lim) ? -INFINITY : s[qb][kb][r];
            }
          }
        }
        // row max: four independent 8-value chains of v_max3, then one combine
        float mx4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x16& a = s[qb][j >> 1];
          const int r0 = (j & 1) * 8;
          float x = max3f(a[r0], a[r0 + 1], a[r0 + 2]);
          x = max3f(x, a[r0 + 3], a[r0 + 4]);
          x = max3f(x, a[r0 + 5], a[r0 + 6]);
          mx4[j] = max3f(x, a[r0 + 7], m[qb]);
        }
        float mx = max3f(mx4[0], mx4[1], max3f(mx4[2], mx4[3], m[qb]));
        mx = half_max(mx);
        // deferred rescale (see attn_fwd_kernel): the running max moves only when some row
        // of the block grew by more than 2^8
        alpha[qb] = 1.f;
        if (__any((mx - m[qb]) * c > 8.f)) {
          alpha[qb] = __builtin_amdgcn_exp2f((m[qb] - mx) * c);
          m[qb] = mx;
#pragma unroll
          for (int db = 0; db < NDB; ++db)
#pragma unroll
            for (int r = 0; r < 16; ++r) oacc[qb][db][r] *= alpha[qb];
        }
        const float mc = m[qb] * c;
        float ps4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float e = __builtin_amdgcn_exp2f(fmaf(s[qb][kb][8 * s2 + j], c, -mc));
              ps4[j & 3] = addf(ps4[j & 3], e);
              pf[qb][kb * 2 + s2][j] = f2bf(e);
            }
        lsum[qb] = fmaf(lsum[qb], alpha[qb], addf(addf(ps4[0], ps4[1]), addf(ps4[2], ps4[3])));
      }
      stamp(2);
      mfma_prio(true);
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        bf16x8 vfr[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) vfr[kk] = tr_frag<D>(Vs, kk * 16 + 4 * h32, db * 32, lane, 8);
#pragma unroll
        for (int qb = 0; qb < QB; ++qb)
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) oacc[qb][db] = mfma32(vfr[kk], pf[qb][kk], oacc[qb][db]);
      }
      mfma_prio(false);
      stamp(3);
    }
    stamp(-1);
    __syncthreads();
    stamp(4);
  };

  gload(0);
  swrite(std::integral_constant<int, 0>{});
  // retire every prologue load (Q fragments included) with a wait the compiler's wait-count
  // pass can see (see attn_fwd_kernel)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  if (ntiles > 1) gload(1);
  __syncthreads();
  stamp(-1);
  st_begin = st_prev;
  for (int t = 0; t < ntiles; t += 2) {
    tile(std::integral_constant<int, 0>{}, t);
    if (t + 1 < ntiles) tile(std::integral_constant<int, 1>{}, t + 1);
  }
  if constexpr (STAMPS) {
    // keep the whole computation alive (the stamped kernel stores no O): a checksum of the
    // accumulators decides a store that never happens
    float chk = 0.f;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      chk += lsum[qb] + m[qb];
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) chk += oacc[qb][db][r];
    }
    if (chk == 1.2345e-30f) p.lse[tid] = chk;
    if (lane == 0) {
      unsigned long long* out = reinterpret_cast<unsigned long long*>(p.o) + ((long)blockIdx.x * 4 + wv) * 8;
      for (int k = 0; k < 5; ++k) out[k] = st_acc[k];
      out[5] = (unsigned long long)st_n;
      out[6] = (unsigned long long)ntiles;
      out[7] = st_prev - st_begin;
    }
    return;
  }

#pragma unroll
  for (int qb = 0; qb < QB; ++qb) {
    const int myq = qw0 + qb * 32 + l32;
    const float lt = half_sum(lsum[qb]);
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
    if (myq < p.T) {
      bf16_t* Ob = p.o + b * p.o_sb + hq * p.o_sh + (long)myq * p.o_st;
#pragma unroll
      for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          bf16x4 v4;
#pragma unroll
          for (int j = 0; j < 4; ++j) v4[j] = f2bf(oacc[qb][db][4 * g4 + j] * inv);
          *reinterpret_cast<bf16x4*>(Ob + db * 32 + 8 * g4 + 4 * h32) = v4;
        }
      if (h32 == 0) p.lse[((long)b * p.Hq + hq) * p.T + myq] = m[qb] * c + __log2f(lt);
    }
  }
}

// ---------------------------------------------------------------------------------------
// attn_fwd4 (round 5, D = 64): four waves per SIMD.  The round-3/4 forward holds 255 VGPRs
// (two 32-row query blocks per wave, K / V staged through registers) and so runs at two waves
// per SIMD, where its per-tile chain (S MFMAs -> row max -> exp -> pack -> PV MFMAs) is
// latency-bound: stamps put half a tile in the softmax phase and a quarter at the barrier
// (docs/PERFORMANCE.md, "Attention").  Here one 32-row block per wave, K / V tiles arrive by
// LDS-DMA (no staging registers), the LDS fragment reads are inline asm with hand-counted
// waits (the compiler's wait-count pass would drain the DMA ring before its own LDS reads),
// and the register diet (Q 16, O 32, S 32 / P 16, one block of K or V fragments 16) keeps the
// kernel under 128 VGPRs: four workgroups of 4 waves per CU (32 KB of LDS each), so every
// SIMD interleaves four waves' chains.  Same algorithm and numerics as attn_fwd3: swapped
// S^T = K Q^T with the query on the lane, online softmax in base 2 with the deferred rescale,
// P from the accumulators into O^T += V^T P^T.
template <bool CAUSAL>
__global__ __launch_bounds__(256, 4) void attn_fwd4_kernel(AttnParams p) {
  constexpr int D = 64, BM = 128, BN = 64, TILE = BN * D;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];  // [2 bufs][K|V][TILE]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h32 = lane >> 5, l32 = lane & 31;
  const int BH = p.B * p.Hq;
  const int nqt = (p.T + BM - 1) / BM;
  const int bh = blockIdx.x % BH;
  const int qt = nqt - 1 - (int)(blockIdx.x / BH);  // heaviest (causal) tiles launch first
  const int b = bh / p.Hq, hq = bh % p.Hq, hk = hq / (p.Hq / p.Hkv);
  const int q0 = qt * BM, qw0 = q0 + wv * 32;
  const int off = p.Tk - p.T;  // causal: key <= query + off
  const float c = p.scale_log2;

  const bf16_t* Qb = p.q + b * p.q_sb + hq * p.q_sh;
  const bf16_t* Kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* Vb = p.v + b * p.v_sb + hk * p.v_sh;

  bf16x8 qf[D / 16];
  {
    const int qr = min(qw0 + l32, p.T - 1);
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks)
      qf[ks] = *reinterpret_cast<const bf16x8*>(Qb + (long)qr * p.q_st + ks * 16 + 8 * h32);
  }
  const int kend = CAUSAL ? min(p.Tk, q0 + BM + off) : p.Tk;
  const int ntiles = (kend + BN - 1) / BN;

  // LDS-DMA: a tile's K (and V) image is 8 pieces of 8 rows x 128 bytes; wave wv issues
  // pieces 2 wv, 2 wv + 1 of each.  Lane: row 8 pc + lane / 8, physical chunk lane % 8, read
  // from the logical chunk (lane % 8) ^ swz<64>(row) (loff<64>'s XOR, an involution).  Full
  // tiles advance by the scalar offset; a last partial tile clamps its rows to the last key.
  const unsigned kst_b = (unsigned)p.k_st * 2, vst_b = (unsigned)p.v_st * 2;
  const __amdgpu_buffer_rsrc_t rk = make_rsrc(Kb, (unsigned)((long)(p.Tk - 1) * p.k_st + D) * 2);
  const __amdgpu_buffer_rsrc_t rv = make_rsrc(Vb, (unsigned)((long)(p.Tk - 1) * p.v_st + D) * 2);
  const int prow0 = 16 * wv + (lane >> 3);  // piece e adds 8 rows
  auto dma = [&](int t, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    bf16_t* Ks = smem + buf * 2 * TILE;
    const int k0 = t * BN;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int row = prow0 + 8 * e;
      const unsigned ch16 = 16u * (unsigned)((lane & 7) ^ swz<D>(row));
      if (k0 + BN <= p.Tk) {
        blds16(rk, (unsigned)row * kst_b + ch16, (unsigned)k0 * kst_b, Ks + (2 * wv + e) * 512);
        blds16(rv, (unsigned)row * vst_b + ch16, (unsigned)k0 * vst_b, Ks + TILE + (2 * wv + e) * 512);
      } else {
        const unsigned key = (unsigned)min(k0 + row, p.Tk - 1);
        blds16(rk, key * kst_b + ch16, 0, Ks + (2 * wv + e) * 512);
        blds16(rv, key * vst_b + ch16, 0, Ks + TILE + (2 * wv + e) * 512);
      }
    }
  };
  // per-lane LDS byte bases: K rows l32 (d chunk 2 ks + h32: four bases, the key block by an
  // immediate); V transposed reads of key rows kk 16 + 4 h32 + (iq >> 2) (+ 8: second half),
  // columns db 32 + 16 (gq & 1) + 4 (iq & 3) -- the swizzle does not depend on kk, so one base
  // per (db, half) and kk by an immediate
  const unsigned lds0 = lds_addr(smem, 0);
  unsigned kad[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) kad[ks] = lds0 + 2u * (unsigned)loff<D>(l32, ks * 16 + 8 * h32);
  const int gq = lane >> 4, iq = lane & 15;
  unsigned vad[2][2];
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
      vad[db][hf] = lds0 + 2u * (unsigned)(TILE + loff<D>(4 * h32 + (iq >> 2) + 8 * hf, db * 32 + 16 * (gq & 1) + 4 * (iq & 3)));

  f32x16 oacc[2];
  oacc[0] = zero16();
  oacc[1] = zero16();
  float m = -1e30f, lsum = 0.f;

  auto tile = [&](int t, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    constexpr unsigned BOFF = buf * 2 * TILE * 2;  // bytes
    // tile t landed (this wave's pieces; the barrier: everyone's) and every wave is done with
    // the other buffer (read in tile t - 1): tile t + 1 may overwrite it
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < ntiles) dma(t + 1, std::integral_constant<int, buf ^ 1>{});
    const int k0 = t * BN;
    const bool active = !CAUSAL || (k0 <= qw0 + 31 + off);
    if (!active) return;
    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      bf16x8 kf[D / 16];
      if (kb == 0) {
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) kf[ks] = b128_read_at<BOFF>(kad[ks]);
      } else {
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) kf[ks] = b128_read_at<BOFF + 32 * D * 2>(kad[ks]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(kf[0]), "+v"(kf[1]), "+v"(kf[2]), "+v"(kf[3]));
      s[kb] = zero16();
      mfma_prio(true);
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) s[kb] = mfma32(kf[ks], qf[ks], s[kb]);
      mfma_prio(false);
    }
    const bool need_mask = (CAUSAL && (k0 + BN - 1 > qw0 + off)) || (k0 + BN > p.Tk);
    if (need_mask) {
      const int vis = CAUSAL ? min(qw0 + l32 + off, p.Tk - 1) : p.Tk - 1;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const int lim = vis - (k0 + kb * 32 + 4 * h32);
#pragma unroll
        for (int r = 0; r < 16; ++r) s[kb][r] = ((r & 3) + 8 * (r >> 2) > lim) ? -INFINITY : s[kb][r];
      }
    }
    float mx4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x16& a = s[j >> 1];
      const int r0 = (j & 1) * 8;
      float x = max3f(a[r0], a[r0 + 1], a[r0 + 2]);
      x = max3f(x, a[r0 + 3], a[r0 + 4]);
      x = max3f(x, a[r0 + 5], a[r0 + 6]);
      mx4[j] = max3f(x, a[r0 + 7], m);
    }
    float mx = max3f(mx4[0], mx4[1], max3f(mx4[2], mx4[3], m));
    mx = half_max(mx);
    float alpha = 1.f;
    if (__any((mx - m) * c > 8.f)) {
      alpha = __builtin_amdgcn_exp2f((m - mx) * c);
      m = mx;
#pragma unroll
      for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int r = 0; r < 16; ++r) oacc[db][r] *= alpha;
    }
    const float mc = m * c;
    float ps4[4] = {0.f, 0.f, 0.f, 0.f};
    bf16x8 pf[4];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float e = __builtin_amdgcn_exp2f(fmaf(s[kb][8 * s2 + j], c, -mc));
          ps4[j & 3] = addf(ps4[j & 3], e);
          pf[kb * 2 + s2][j] = f2bf(e);
        }
    lsum = fmaf(lsum, alpha, addf(addf(ps4[0], ps4[1]), addf(ps4[2], ps4[3])));
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      // V^T fragments: two transposed 4-row reads each, kept as halves until their wait
      bf16x4 vlo[4], vhi[4];
      vlo[0] = tr_read_at<BOFF + 0 * 16 * D * 2>(vad[db][0]);
      vhi[0] = tr_read_at<BOFF + 0 * 16 * D * 2>(vad[db][1]);
      vlo[1] = tr_read_at<BOFF + 1 * 16 * D * 2>(vad[db][0]);
      vhi[1] = tr_read_at<BOFF + 1 * 16 * D * 2>(vad[db][1]);
      vlo[2] = tr_read_at<BOFF + 2 * 16 * D * 2>(vad[db][0]);
      vhi[2] = tr_read_at<BOFF + 2 * 16 * D * 2>(vad[db][1]);
      vlo[3] = tr_read_at<BOFF + 3 * 16 * D * 2>(vad[db][0]);
      vhi[3] = tr_read_at<BOFF + 3 * 16 * D * 2>(vad[db][1]);
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(vlo[0]), "+v"(vlo[1]), "+v"(vlo[2]), "+v"(vlo[3]), "+v"(vhi[0]), "+v"(vhi[1]),
                     "+v"(vhi[2]), "+v"(vhi[3]));
      mfma_prio(true);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) oacc[db] = mfma32(cat8(vlo[kk], vhi[kk]), pf[kk], oacc[db]);
      mfma_prio(false);
    }
  };

  dma(0, std::integral_constant<int, 0>{});
  for (int t = 0; t < ntiles; t += 2) {
    tile(t, std::integral_constant<int, 0>{});
    if (t + 1 < ntiles) tile(t + 1, std::integral_constant<int, 1>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA in flight when the workgroup ends

  const int myq = qw0 + l32;
  const float lt = half_sum(lsum);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (myq < p.T) {
    bf16_t* Ob = p.o + b * p.o_sb + hq * p.o_sh + (long)myq * p.o_st;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        bf16x4 v4;
#pragma unroll
        for (int j = 0; j < 4; ++j) v4[j] = f2bf(oacc[db][4 * g4 + j] * inv);
        *reinterpret_cast<bf16x4*>(Ob + db * 32 + 8 * g4 + 4 * h32) = v4;
      }
    if (h32 == 0) p.lse[((long)b * p.Hq + hq) * p.T + myq] = m * c + __log2f(lt);
  }
}

}  // namespace orion

using namespace orion;

extern "C++" {

template <int D, bool CAUSAL, int QB>
static void fwd3_attr() {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)attn_fwd3_kernel<D, CAUSAL, QB>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 2 * 64 * D * 2);
    done = true;
  }
}

template <bool CAUSAL>
static void fwd4_launch(const AttnParams& p, hipStream_t st) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)attn_fwd4_kernel<CAUSAL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * 2 * 64 * 64 * 2);
    done = true;
  }
  attn_fwd4_kernel<CAUSAL><<<((p.T + 127) / 128) * p.B * p.Hq, 256, 2 * 2 * 64 * 64 * 2, st>>>(p);
}

// ORION_ATTN_FWD=v3: the D = 64 forward of rounds 3-4 (A/B); default attn_fwd4
static bool fwd_v3() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ORION_ATTN_FWD");
    v = (e && e[0] == 'v' && e[1] == '3') ? 1 : 0;
  }
  return v == 1;
}

template <int D, bool CAUSAL>
static void fwd3_launch(const AttnParams& p, int qb64, size_t lds, hipStream_t st) {
  if constexpr (D == 64 && CAUSAL) {
    static const bool diag = getenv("ORION_ATTN_FWD_DIAG") && getenv("ORION_ATTN_FWD_DIAG")[0] == '1';
    if (diag) {  // stamped instantiation: phase sums over p.o (scripts/attn_fwd_stamps.py)
      (void)hipFuncSetAttribute((const void*)attn_fwd3_kernel<64, true, 2, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 2 * 64 * D * 2);
      attn_fwd3_kernel<64, true, 2, true><<<((p.T + 255) / 256) * p.B * p.Hq, 256, lds, st>>>(p);
      return;
    }
  }
  if constexpr (D == 64) {
    static const bool diag = getenv("ORION_ATTN_FWD_DIAG") && getenv("ORION_ATTN_FWD_DIAG")[0] == '1';
    if constexpr (CAUSAL) {  // the non-causal form runs out of registers at 4 waves: fwd3
      if (!diag && !fwd_v3()) {
        fwd4_launch<CAUSAL>(p, st);
        return;
      }
    }
  }
  if constexpr (D == 64) {
    if (qb64 == 2) {
      fwd3_attr<D, CAUSAL, 2>();
      attn_fwd3_kernel<D, CAUSAL, 2><<<((p.T + 255) / 256) * p.B * p.Hq, 256, lds, st>>>(p);
      return;
    }
  }
  fwd3_attr<D, CAUSAL, 1>();
  attn_fwd3_kernel<D, CAUSAL, 1><<<((p.T + 127) / 128) * p.B * p.Hq, 256, lds, st>>>(p);
}

// returns -1 for an unsupported head dim, -2 when the buffer-offset range is exceeded
// (the caller falls back to the older kernel)
int orion_attn_fwd3(const AttnParams& p, int D, bool causal, hipStream_t st) {
  const long kbytes = ((long)(p.Tk - 1) * p.k_st + D) * 2, vbytes = ((long)(p.Tk - 1) * p.v_st + D) * 2;
  if (kbytes >= (1L << 31) || vbytes >= (1L << 31)) return -2;
  const size_t lds = (size_t)2 * 2 * 64 * D * 2;
  // D = 64: two 32-row query blocks per wave (one K / V fragment read for both, the two
  // softmax chains interleaved with each other's MFMAs; 255 VGPRs) -- equal in isolation to one
  // block per wave but faster in the whole GPT-2 step in 8 of 8 alternating pairs on two boxes
  // (+0.2-0.6 %, profiles/ab/ab_fwd_qb*.log); D = 128: one block per wave.
  constexpr int qb64 = ATTN_FWD_QB64;
#define FWD3(DD, CC) fwd3_launch<DD, CC>(p, qb64, lds, st);
  if (D == 64) {
    if (causal) { FWD3(64, true) } else { FWD3(64, false) }
  } else if (D == 128) {
    if (causal) { FWD3(128, true) } else { FWD3(128, false) }
  } else {
    return -1;
  }
#undef FWD3
  return (int)hipGetLastError();
}

}  // extern "C++"
