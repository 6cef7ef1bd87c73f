// Flash-attention backward as two atomic-free kernels (gfx950): dK/dV with the KEY on the
// lane, dQ with the QUERY on the lane.  Deterministic (every output element is produced
// by one workgroup in a fixed order) and the default backward: faster than the fused
// kernels of attention.hip (one pass producing dK, dV and fp32-atomic dQ partials) at both
// head dims -- at D = 128 those run out of registers (a fused 8-wave / 256-key form needs
// ~370 VGPRs per lane; the 4-wave v1 form runs at one wave per SIMD with the dQ fold
// through LDS on the critical path), at D = 64 the dQ atomics floor them.
//
// The split recomputes S and dP once more (7 instead of 5 matmuls per (q, key) pair) but
// each kernel keeps its accumulators and operand fragments in registers:
//
//   delta          delta[q] = sum_d dO O: written by the dQ kernel's prologue (attn_bwd_dq4 at
//                  D = 64, with the QKV bias also the K / V bias columns; attn_bwd_dq<FD> at
//                  D = 128), so dQ is launched FIRST and dK/dV, which reads delta, after it on
//                  the same stream.  ORION_ATTN_DQ=v3 / ORION_ATTN_DELTA=pass: a separate
//                  HBM-bound pass (attn_delta_kernel) ahead of both kernels.
//   kv kernel      per workgroup 32*NW keys, loop over 32-row query tiles (and the query
//                  heads of its KV head):  S = Q K^T, dP = dO V^T (key on the lane, V
//                  fragments in registers, K in registers or an LDS image),
//                  P = exp2(c S - lse), dS = P (dP - delta),
//                  dV^T += dO^T P, dK^T += Q^T dS (S/dP accumulators reused as B operands)
//   dq kernel      the forward's structure: per workgroup 128 queries (32 per wave), K/V
//                  tiles of 64 keys double-buffered in LDS; S^T = K Q^T and dP^T = V dO^T
//                  (query on the lane: lse and delta are per-lane scalars), dS^T in place,
//                  dQ^T += K^T dS^T with K^T by transposed LDS reads (ds_read_b64_tr_b16),
//                  bf16 dQ written once -- no fp32 accumulator, no conversion pass.
//
// MFMA v_mfma_f32_32x32x16_bf16 throughout; LDS images and fragment helpers: mfma_lds.h.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "common.h"
#include "attn_params.h"
#include "mfma_lds.h"

namespace orion {

// delta[b][h][t] = sum_d dO * O (D/8 lanes per row, 8 bf16 per lane)
//
// BIAS (packed self-attention, Hq == Hkv, D = 64, T % 32 == 0: a workgroup's 32 rows are one
// 32-token block of one head): also the QKV bias gradient's K and V column sums of the block.
// Softmax is invariant to a shift of every key, so sum_keys dK = scale sum_q Q (sum_k dS) = 0
// (sum_k P (dP - delta) = delta - delta); and sum_keys dV = sum_q dO (sum_k P) = sum_q dO.
// The K columns get 0 and the V columns the block's column sum of dO: the dK/dV kernel
// needs no reduction of its own.
template <int D, bool BIAS = false>
__global__ __launch_bounds__(256) void attn_delta_kernel(AttnParams p, float* __restrict__ delta) {
  constexpr int TPR = D / 8;
  const long row = (blockIdx.x * 256L + threadIdx.x) / TPR;
  const int sub = threadIdx.x % TPR;
  const long nrows = (long)p.B * p.Hq * p.T;
  float s = 0.f;
  [[maybe_unused]] bf16x8 d;
  if (row < nrows) {
    const long t = row % p.T, h = (row / p.T) % p.Hq, b = row / ((long)p.T * p.Hq);
    const bf16x8 o = *reinterpret_cast<const bf16x8*>(p.o + b * p.o_sb + h * p.o_sh + t * p.o_st + sub * 8);
    d = *reinterpret_cast<const bf16x8*>(p.dout + b * p.do_sb + h * p.do_sh + t * p.do_st + sub * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += bf2f(o[j]) * bf2f(d[j]);
  }
#pragma unroll
  for (int o2 = TPR / 2; o2 > 0; o2 >>= 1) s += __shfl_xor(s, o2, 64);
  if (row < nrows && sub == 0) delta[row] = s;
  if constexpr (BIAS) {
    static_assert(D == 64, "one 32-row block per workgroup");
    __shared__ float red[32][D + 1];
    const int r = threadIdx.x / TPR;
#pragma unroll
    for (int j = 0; j < 8; ++j) red[r][sub * 8 + j] = row < nrows ? bf2f(d[j]) : 0.f;
    __syncthreads();
    const long row0 = blockIdx.x * 32L;  // first row of the block: (b, h, t0), t0 % 32 == 0
    if (row0 < nrows && threadIdx.x < 2 * D) {
      const long t0 = row0 % p.T, h = (row0 / p.T) % p.Hq, b = row0 / ((long)p.T * p.Hq);
      float* prow = p.bias_part + (b * (p.T / 32) + t0 / 32) * p.bias_ld + (p.Hq + h) * D;
      const int c = threadIdx.x & (D - 1);
      if (threadIdx.x < D) {
        prow[c] = 0.f;  // K columns
      } else {
        float cs = 0.f;
#pragma unroll 8
        for (int i = 0; i < 32; ++i) cs += red[i][c];
        prow[p.Hkv * D + c] = cs;  // V columns
      }
    }
  }
}

// 16 bytes per lane by a raw buffer load (scalar soffset carries the tile position)
ORION_DEVICE bf16x8 bwd_buf_load16(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// Column sums over a wave's 32 rows (lane l32 = row, h32 = d half) of the NDB f32x16
// accumulators x * sc: d = 32 db + (r & 3) + 8 (r >> 2) + 4 h32.  Five halving exchange steps
// over the lane bits (at offset o a lane keeps the half of its live values selected by bit o
// of l32 and adds its partner's copy of it): 31 shuffles for 32 values instead of a
// butterfly per value.  Lane l32 ends with values l32 * (NV / 32) + j, written to
// dst[d(value)]; rows past the end contribute 0 (valid = false).
// The halving exchange of wave_colsum_store on NV values per lane (NV a multiple of 32):
// afterwards v[j] (j < NV / 32) holds the sum over the 32 lanes of one h32 half of value index
// l32 * (NV / 32) + j.
template <int NV>
ORION_DEVICE void wave_colsum_vals(float (&v)[NV], int l32) {
  auto step = [&](auto Oc, auto Lc) {
    constexpr int o = decltype(Oc)::value, L = decltype(Lc)::value, half = L / 2;
    const bool up = (l32 & o) != 0;
#pragma unroll
    for (int k = 0; k < half; ++k) {
      const float send = up ? v[k] : v[half + k];
      const float keep = up ? v[half + k] : v[k];
      v[k] = keep + __shfl_xor(send, o);
    }
  };
  step(std::integral_constant<int, 16>(), std::integral_constant<int, NV>());
  step(std::integral_constant<int, 8>(), std::integral_constant<int, NV / 2>());
  step(std::integral_constant<int, 4>(), std::integral_constant<int, NV / 4>());
  step(std::integral_constant<int, 2>(), std::integral_constant<int, NV / 8>());
  step(std::integral_constant<int, 1>(), std::integral_constant<int, NV / 16>());
}

template <int NDB>
ORION_DEVICE void wave_colsum_store(const f32x16 (&x)[NDB], float sc, bool valid, int l32, int h32,
                                    float* __restrict__ dst) {
  constexpr int NV = 16 * NDB;
  float v[NV];
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) v[16 * db + r] = valid ? x[db][r] * sc : 0.f;
  wave_colsum_vals<NV>(v, l32);
#pragma unroll
  for (int j = 0; j < NV / 32; ++j) {
    const int idx = l32 * (NV / 32) + j, db = idx >> 4, r = idx & 15;
    dst[32 * db + (r & 3) + 8 * (r >> 2) + 4 * h32] = v[j];
  }
}

// Store one lane's row of a dK / dQ accumulator set (lane = token, registers = d: d = 32 db +
// (r & 3) + 8 (r >> 2) + 4 h32) as bf16, times `sc`; with rope tables, the inverse rotation
// (rotate-half pairs d, d + D/2 = accumulators db, db + NDB/2 at the same r): the gradient
// w.r.t. the unrotated input, dx1 = c g1 + s g2, dx2 = c g2 - s g1.
template <int NDB>
ORION_DEVICE void store_row_grad(const f32x16 (&acc)[NDB], float sc, bf16_t* __restrict__ dst, int h32,
                                 const float* __restrict__ rc, const float* __restrict__ rs) {
  constexpr int D = 32 * NDB, H = NDB / 2;
  if (rc) {
#pragma unroll
    for (int db = 0; db < H; ++db)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int d = db * 32 + 8 * g4 + 4 * h32;
        const f32x4 c = *reinterpret_cast<const f32x4*>(rc + d), sn = *reinterpret_cast<const f32x4*>(rs + d);
        bf16x4 lo, hi;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float g1 = acc[db][4 * g4 + j] * sc, g2 = acc[db + H][4 * g4 + j] * sc;
          lo[j] = f2bf(c[j] * g1 + sn[j] * g2);
          hi[j] = f2bf(c[j] * g2 - sn[j] * g1);
        }
        *reinterpret_cast<bf16x4*>(dst + d) = lo;
        *reinterpret_cast<bf16x4*>(dst + d + D / 2) = hi;
      }
    return;
  }
#pragma unroll
  for (int db = 0; db < NDB; ++db)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      bf16x4 v4;
#pragma unroll
      for (int j = 0; j < 4; ++j) v4[j] = f2bf(acc[db][4 * g4 + j] * sc);
      *reinterpret_cast<bf16x4*>(dst + db * 32 + 8 * g4 + 4 * h32) = v4;
    }
}

// ============================================================================ dK / dV
// NW waves x 32 keys per workgroup; query tiles of 32 rows double-buffered in LDS
// (register staged: the next tile's loads are issued before this tile's MFMAs and written
// after them).  One LDS barrier per tile.  Two workgroups per CU (two waves per SIMD, so
// one wave's MFMAs overlap the other's softmax / LDS phase): at D = 128 that fits the
// 256-register budget only with the K fragments read from an LDS image per query tile
// (KLDS) instead of held in registers (25 spilled registers otherwise).
template <int D>
__host__ __device__ constexpr int kv_waves() { return 4; }

// STAMPS (diagnostic instantiation, ORION_ATTN_DIAG=1, D = 64): every wave accumulates
// s_memtime deltas of the five phases of a query tile (S/dP chain issue, softmax, dV/dK
// issue, LDS stage write, barrier) and writes them with its active-tile count and lifetime
// over p.dq (the dQ kernel is then skipped): scripts/attn_stamps.py, profiles/attn_r03/.
template <int D, bool CAUSAL, bool STAMPS = false>
__global__ __launch_bounds__(kv_waves<D>() * 64, 2) void attn_bwd_kv_kernel(AttnParams p) {
  constexpr int NW = kv_waves<D>(), NT = NW * 64;
  constexpr int BNK = 32 * NW, BMQ = 32, NCH = D / 8, NDB = D / 32;
  constexpr int QT = BMQ * D;            // Q / dO tile elements
  constexpr int NQC = BMQ * NCH;         // 16-byte chunks per Q (or dO) tile
  constexpr int NSTQ = 2 * NQC / NT;     // chunks per thread per Q+dO stage
  constexpr bool KLDS = D == 128;        // K fragments from an LDS image, not registers
  static_assert(NSTQ >= 1 && NSTQ * NT == 2 * NQC, "Q/dO staging must divide over the threads");
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  bf16_t* Ks = smem;                                        // [BNK][D] (KLDS only)
  bf16_t* Qs = Ks + (KLDS ? BNK * D : 0);                   // [2][32][D]
  bf16_t* Ds = Qs + 2 * QT;                                 // [2][32][D] (dO)
  float* lse_s = reinterpret_cast<float*>(Ds + 2 * QT);     // [2][32]  -lse / c
  float* del_s = lse_s + 2 * BMQ;                           // [2][32]  -delta

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h32 = lane >> 5, l32 = lane & 31;
  const int BHk = p.B * p.Hkv;
  const int kt = blockIdx.x / BHk;  // small kt = most work under the causal mask: first
  const int bh = blockIdx.x % BHk;
  const int b = bh / p.Hkv, hk = bh % p.Hkv;
  const int rep = p.Hq / p.Hkv;
  const int kt0 = kt * BNK, kw0 = kt0 + wv * 32, mykey = kw0 + l32;
  const int off = p.Tk - p.T;
  const float c = p.scale_log2, inv_c = 1.f / p.scale_log2;

  const bf16_t* Kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* Vb = p.v + b * p.v_sb + hk * p.v_sh;
  // K / V fragments of this wave's 32 keys: B operands of S and dP for every query tile
  bf16x8 kf[KLDS ? 1 : D / 16], vf[D / 16];
  {
    const long key = min(mykey, p.Tk - 1);
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      if constexpr (!KLDS) kf[ks] = *reinterpret_cast<const bf16x8*>(Kb + key * p.k_st + ks * 16 + 8 * h32);
      vf[ks] = *reinterpret_cast<const bf16x8*>(Vb + key * p.v_st + ks * 16 + 8 * h32);
    }
  }
  if constexpr (KLDS) {
    for (int cidx = tid; cidx < BNK * NCH; cidx += NT) {
      const int row = cidx / NCH, ch = cidx % NCH;
      const long key = min(kt0 + row, p.Tk - 1);
      *reinterpret_cast<bf16x8*>(Ks + loff<D>(row, ch * 8)) =
          *reinterpret_cast<const bf16x8*>(Kb + key * p.k_st + ch * 8);
    }
  }
  f32x16 dka[NDB], dva[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db) { dka[db] = zero16(); dva[db] = zero16(); }

  const int qlo = CAUSAL ? max(0, kt0 - off) : 0;  // first query row that sees any key here
  const int qi0 = qlo / BMQ;
  const int nqi = (p.T + BMQ - 1) / BMQ;
  const int iters_per_head = max(0, nqi - qi0);
  const int total = iters_per_head * rep;

  bf16x8 qdst[NSTQ];
  float lse_r = 0.f, del_r = 0.f;
  // Q / dO tiles by buffer loads over this batch's rows of all query heads: one per-thread
  // 32-bit offset (its row / chunk in the tile), the (head, tile) position in the scalar
  // offset; the clamped path runs only for a last partial query tile
  const bf16_t* Qbb = p.q + b * p.q_sb;
  const bf16_t* Dbb = p.dout + b * p.do_sb;
  const __amdgpu_buffer_rsrc_t rq =
      make_rsrc(Qbb, (unsigned)(((long)(p.T - 1) * p.q_st + (long)(p.Hq - 1) * p.q_sh + D) * 2));
  const __amdgpu_buffer_rsrc_t rd =
      make_rsrc(Dbb, (unsigned)(((long)(p.T - 1) * p.do_st + (long)(p.Hq - 1) * p.do_sh + D) * 2));
  constexpr int NQ = NSTQ >= 2 ? NSTQ / 2 : 1;  // chunks per thread per tensor
  unsigned vq[NQ];
  // this thread's tile row / 16-byte chunk for chunk i (recomputed where needed: registers
  // are short at D = 128)
  auto qrow = [&](int i) { return NSTQ >= 2 ? (tid + i * NT) / NCH : (tid - (tid >= NQC) * NQC) / NCH; };
  auto qch = [&](int i) { return NSTQ >= 2 ? (tid + i * NT) % NCH : (tid - (tid >= NQC) * NQC) % NCH; };
  const bool isd = NSTQ < 2 && tid >= NQC;
  const unsigned qst_b = (unsigned)(isd ? p.do_st : p.q_st) * 2, dst_b = (unsigned)p.do_st * 2;
#pragma unroll
  for (int i = 0; i < NQ; ++i) vq[i] = qrow(i) * (NSTQ >= 2 ? (unsigned)p.q_st * 2 : qst_b) + qch(i) * 16;
  unsigned vdo[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) vdo[i] = qrow(i) * dst_b + qch(i) * 16;
  // chunk i > 0 sits RSTEP rows below chunk 0 (same column): its load offset differs by a
  // wave-uniform amount (carried in the scalar offset) and, the swizzle repeating every 16
  // rows, its LDS offset by a constant -- one offset register per tensor instead of NQ (at
  // D = 128 the kernel is at 256 VGPRs and the extra offsets were spilled, their reload
  // waiting vmcnt(0) in front of every step's Q / dO load issue)
  constexpr int RSTEP = NT / NCH;
  constexpr bool ONEOFF = NSTQ >= 2 && RSTEP % 16 == 0;
  const unsigned qstep = (unsigned)RSTEP * p.q_st * 2, dstep = (unsigned)RSTEP * p.do_st * 2;
  auto gload = [&](int h, int qi) {
    const int hq = hk * rep + h;
    const int qbase = qi * BMQ;
    const unsigned sq = (unsigned)((long)hq * p.q_sh + (long)qbase * p.q_st) * 2;
    const unsigned sd = (unsigned)((long)hq * p.do_sh + (long)qbase * p.do_st) * 2;
    if (qbase + BMQ <= p.T) {
      if constexpr (NSTQ >= 2) {
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
          qdst[i] = bwd_buf_load16(rq, ONEOFF ? vq[0] : vq[i], ONEOFF ? sq + i * qstep : sq);
          qdst[NQ + i] = bwd_buf_load16(rd, ONEOFF ? vdo[0] : vdo[i], ONEOFF ? sd + i * dstep : sd);
        }
      } else {
        qdst[0] = isd ? bwd_buf_load16(rd, vq[0], sd) : bwd_buf_load16(rq, vq[0], sq);
      }
    } else {  // rows past T re-read the last query row (masked in the step)
      const unsigned sq0 = (unsigned)((long)hq * p.q_sh) * 2, sd0 = (unsigned)((long)hq * p.do_sh) * 2;
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const unsigned q = (unsigned)min(qbase + qrow(i), p.T - 1);
        if constexpr (NSTQ >= 2) {
          qdst[i] = bwd_buf_load16(rq, q * (unsigned)p.q_st * 2 + qch(i) * 16, sq0);
          qdst[NQ + i] = bwd_buf_load16(rd, q * dst_b + qch(i) * 16, sd0);
        } else {
          qdst[0] = isd ? bwd_buf_load16(rd, q * dst_b + qch(0) * 16, sd0)
                        : bwd_buf_load16(rq, q * (unsigned)p.q_st * 2 + qch(0) * 16, sq0);
        }
      }
    }
    if (tid < BMQ) {
      const long q = min(qbase + tid, p.T - 1);
      const long r = ((long)b * p.Hq + hq) * p.T + q;
      lse_r = p.lse[r];
      del_r = p.delta[r];
    }
  };
  int qlo_[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) qlo_[i] = loff<D>(qrow(i), qch(i) * 8);
  auto swrite = [&](int buf) {
    if constexpr (NSTQ >= 2) {
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const int lo = ONEOFF ? qlo_[0] + i * RSTEP * D : qlo_[i];
        *reinterpret_cast<bf16x8*>(Qs + buf * QT + lo) = qdst[i];
        *reinterpret_cast<bf16x8*>(Ds + buf * QT + lo) = qdst[NQ + i];
      }
    } else {
      *reinterpret_cast<bf16x8*>((isd ? Ds : Qs) + buf * QT + qlo_[0]) = qdst[0];
    }
    if (tid < BMQ) {  // row constants as the initial S / dP accumulators
      lse_s[buf * BMQ + tid] = -lse_r * inv_c;
      del_s[buf * BMQ + tid] = -del_r;
    }
  };

  int nh = 0, nq = qi0;  // next tile to load
  auto advance = [&](int& h, int& qi) {
    if (++qi == nqi) { qi = qi0; ++h; }
  };
  if (total > 0) {
    gload(nh, nq);
    advance(nh, nq);
    swrite(0);
  }
  // Retire the K / V fragment loads (and the prologue's) with a wait the compiler's wait-count
  // pass can see on every path.  Without it the pass, merging the total == 0 path at the
  // loop, left vmcnt waits for kf / vf in front of the S / dP MFMAs of EVERY step -- and in
  // the steady state those counted waits drained the next step's Q / dO prefetch, so each
  // step's MFMA chain sat out the full load latency (round 3's stamps: ~1,290 cycles in the
  // S / dP chain, ~1,760 at the stage write).
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
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
  stamp(-1);
  st_begin = st_prev;
  int cq = qi0;  // query tile of this step
  for (int it = 0; it < total; ++it) {
    stamp(-1);
    const int buf = it & 1;
    const int qbase = cq * BMQ;
    if (++cq == nqi) cq = qi0;
    if (it + 1 < total) {
      gload(nh, nq);
      advance(nh, nq);
    }
    const bf16_t* Qc = Qs + buf * QT;
    const bf16_t* Dc = Ds + buf * QT;
    // wave-uniform: this wave's keys are all above every query of the tile
    const bool active = !CAUSAL || (qbase + BMQ - 1 + off >= kw0);
    if (active) {
      // S - lse/c and dP - delta straight out of the MFMA chains (row constants preloaded)
      f32x16 s, dp;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 L = *reinterpret_cast<const f32x4*>(lse_s + buf * BMQ + 8 * g4 + 4 * h32);
        const f32x4 Dl = *reinterpret_cast<const f32x4*>(del_s + buf * BMQ + 8 * g4 + 4 * h32);
#pragma unroll
        for (int j = 0; j < 4; ++j) { s[4 * g4 + j] = L[j]; dp[4 * g4 + j] = Dl[j]; }
      }
      // D = 128: the per-fragment LDS offsets are rebuilt each step from one opaque per-lane
      // base (one xor per read) instead of being held as 16 loop-invariant
      // registers -- at 256 VGPRs those pushed V fragments / offsets into scratch, and each
      // reload waited vmcnt(0) behind the step's Q / dO prefetch.  Column chunk 2 ks + h32 of
      // row l32 sits at chunk (2 ks) ^ (h32 ^ swz(l32)); rows wv * 32 + l32 of the K image
      // share the swizzle of row l32 (period 16).
      int zb = (l32 * D) | ((h32 ^ swz<D>(l32)) << 3);
      if constexpr (KLDS) asm volatile("" : "+v"(zb));
      const bf16_t* Kw = Ks + wv * 32 * D;
      mfma_prio(true);
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        const int o = KLDS ? (zb ^ (ks << 4)) : loff<D>(l32, ks * 16 + 8 * h32);
        bf16x8 kfr;
        if constexpr (KLDS) kfr = lds_b128(Kw, o);
        else kfr = kf[ks];
        s = mfma32(lds_b128(Qc, o), kfr, s);
        dp = mfma32(lds_b128(Dc, o), vf[ks], dp);
        if constexpr (KLDS) { if (ks % 2 == 1) __builtin_amdgcn_sched_barrier(0); }
      }
      mfma_prio(false);
      stamp(0);
      ++st_n;
      // P and dS in place: row q = qbase + (r&3)+8(r>>2)+4*h32, column = mykey
      const bool need_mask = (CAUSAL && (qbase + off < kw0 + 31)) || (kw0 + 32 > p.Tk) ||
                             (qbase + BMQ > p.T);
      if (need_mask) {
        // row q = qbase + rowoff(r) + 4*h32 contributes iff lo <= rowoff(r) < hi
        const int q4 = qbase + 4 * h32;
        const int lo = CAUSAL ? mykey - off - q4 : 0;
        const int hi = mykey < p.Tk ? p.T - q4 : 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          s[r] = (ro < lo || ro >= hi) ? -INFINITY : s[r];
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = __builtin_amdgcn_exp2f(s[r] * c);
        s[r] = pv;
        dp[r] = pv * dp[r];  // dS / scale: the scale is applied to dK once at the end
      }
      bf16x8 pb[2], sb[2];
      pb[0] = acc_to_frag(s, 0);
      pb[1] = acc_to_frag(s, 1);
      sb[0] = acc_to_frag(dp, 0);
      sb[1] = acc_to_frag(dp, 1);
      stamp(1);
      mfma_prio(true);
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          dva[db] = mfma32(tr_frag<D>(Dc, 16 * s2 + 4 * h32, db * 32, lane, 8), pb[s2], dva[db]);
          dka[db] = mfma32(tr_frag<D>(Qc, 16 * s2 + 4 * h32, db * 32, lane, 8), sb[s2], dka[db]);
        }
      }
      mfma_prio(false);
      stamp(2);
    }
    if (it + 1 < total) swrite(buf ^ 1);
    stamp(3);
    __syncthreads();
    stamp(4);
  }
  if constexpr (STAMPS) {
    // keep the computation alive (the stamped kernel stores no dK / dV; without this the
    // compiler drops every MFMA and LDS read -- round 3's stamps timed that gutted kernel)
    float chk = 0.f;
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) chk += dka[db][r] + dva[db][r];
    if (chk == 1.2345e-30f) p.dk[tid] = 0;
    if (lane == 0) {
      unsigned long long* out = reinterpret_cast<unsigned long long*>(p.dq) + ((long)blockIdx.x * NW + wv) * 8;
      for (int k = 0; k < 5; ++k) out[k] = st_acc[k];
      out[5] = (unsigned long long)st_n;
      out[6] = (unsigned long long)total;
      out[7] = st_prev - st_begin;
    }
    return;
  }

  // dK / dV: lane = key, registers = d ((r&3)+8(r>>2)+4*h32)
  if (mykey < p.Tk) {
    bf16_t* dKb = p.dk + b * p.dk_sb + hk * p.dk_sh + (long)mykey * p.dk_st;
    bf16_t* dVb = p.dv + b * p.dv_sb + hk * p.dv_sh + (long)mykey * p.dv_st;
    const long rrow = (long)(mykey + p.rope_pos0) * (D / 2);
    store_row_grad<NDB>(dka, p.scale, dKb, h32, p.rope_cos ? p.rope_cos + rrow : nullptr,
                        p.rope_sin ? p.rope_sin + rrow : nullptr);
    store_row_grad<NDB>(dva, 1.f, dVb, h32, nullptr, nullptr);
  }
}

// ============================================================================ dQ
// One 256-thread workgroup = 4 waves x 32 queries; key tiles of 64 double-buffered in LDS.
// Per-tile bookkeeping as in attn_fwd.hip's forward: K / V staged by buffer loads with the
// tile advance in the scalar offset, the tile loop unrolled over the two LDS buffers (every
// LDS address a per-lane register plus an immediate), the causal / length mask one
// compare + select per score against a per-lane bound.
// FD (fused delta, round 6; the D = 128 default): delta = rowsum(dO O) is computed in the
// prologue from this wave's own query rows and written for the dK/dV kernel, which then runs
// AFTER this one (as attn_bwd_dq4 at D = 64) -- no separate delta pass.
template <int D, bool CAUSAL, bool BIAS = false, bool FD = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(AttnParams p) {
  constexpr int BM = 128, BN = 64, NCH = D / 8, TILE = BN * D, NST = BN * NCH / 256, NDB = D / 32;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];  // [2 bufs][K|V][TILE]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h32 = lane >> 5, l32 = lane & 31;
  const int BH = p.B * p.Hq;
  const int nqt = (p.T + BM - 1) / BM;
  const int bh = blockIdx.x % BH;
  const int qt = nqt - 1 - (int)(blockIdx.x / BH);  // heaviest (causal) tiles launch first
  const int b = bh / p.Hq, hq = bh % p.Hq, hk = hq / (p.Hq / p.Hkv);
  const int q0 = qt * BM, qw0 = q0 + wv * 32, myq = qw0 + l32;
  const int off = p.Tk - p.T;
  const float c = p.scale_log2;

  const bf16_t* Kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* Vb = p.v + b * p.v_sb + hk * p.v_sh;

  // Q and dO fragments of this wave's 32 queries: B operands of S^T = K Q^T, dP^T = V dO^T
  bf16x8 qf[D / 16], df[D / 16];
  float L, dl;
  {
    const int qr = min(myq, p.T - 1);
    const bf16_t* Qr = p.q + b * p.q_sb + hq * p.q_sh + (long)qr * p.q_st;
    const bf16_t* Dr = p.dout + b * p.do_sb + hq * p.do_sh + (long)qr * p.do_st;
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      qf[ks] = *reinterpret_cast<const bf16x8*>(Qr + ks * 16 + 8 * h32);
      df[ks] = *reinterpret_cast<const bf16x8*>(Dr + ks * 16 + 8 * h32);
    }
    const long r = ((long)b * p.Hq + hq) * p.T + qr;
    L = p.lse[r];
    if constexpr (FD) {
      const bf16_t* Or = p.o + b * p.o_sb + hq * p.o_sh + (long)qr * p.o_st;
      float d4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        const bf16x8 of = *reinterpret_cast<const bf16x8*>(Or + ks * 16 + 8 * h32);
#pragma unroll
        for (int j = 0; j < 8; ++j) d4[j & 3] = fmaf(bf2f(of[j]), bf2f(df[ks][j]), d4[j & 3]);
      }
      dl = (d4[0] + d4[1]) + (d4[2] + d4[3]);
      dl += __shfl_xor(dl, 32);  // the other d half of the row
      if (h32 == 0 && myq < p.T) const_cast<float*>(p.delta)[r] = dl;  // read by the dK/dV kernel
    } else {
      dl = p.delta[r];
    }
  }
  const int kend = CAUSAL ? min(p.Tk, q0 + BM + off) : p.Tk;
  const int ntiles = (kend + BN - 1) / BN;

  const unsigned kst_b = (unsigned)p.k_st * 2, vst_b = (unsigned)p.v_st * 2;
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
        kst[i] = bwd_buf_load16(rk, vk[i], sk);
        vst[i] = bwd_buf_load16(rv, vv[i], sv);
      }
    } else {  // last partial tile: rows past Tk re-read the last key (masked below)
#pragma unroll
      for (int i = 0; i < NST; ++i) {
        const int cidx = tid + i * 256, row = cidx / NCH, ch = cidx % NCH;
        const unsigned key = (unsigned)min(t * BN + row, p.Tk - 1);
        kst[i] = bwd_buf_load16(rk, key * kst_b + ch * 16, 0);
        vst[i] = bwd_buf_load16(rv, key * vst_b + ch * 16, 0);
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
  int ko[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) ko[ks] = loff<D>(l32, ks * 16 + 8 * h32);
  // key k0 + rowoff(r) + 4*h32 of a 32-key block is visible to this lane's query iff
  // rowoff(r) <= vis - k0 - 4*h32
  const int vis = (CAUSAL ? min(myq + off, p.Tk - 1) : p.Tk - 1) - 4 * h32;

  f32x16 dq[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db) dq[db] = zero16();

  auto tile = [&](auto bufc, int t) {
    constexpr int buf = decltype(bufc)::value;
    if (t + 1 < ntiles) gload(t + 1);
    const bf16_t* Ks = smem + buf * 2 * TILE;
    const bf16_t* Vs = Ks + TILE;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const int k0 = t * BN + kb * 32;
      if (CAUSAL && k0 > qw0 + 31 + off) continue;  // wave-uniform: block fully masked
      f32x16 s = zero16(), dp = zero16();
      mfma_prio(true);
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        s = mfma32(lds_b128(Ks + kb * 32 * D, ko[ks]), qf[ks], s);
        dp = mfma32(lds_b128(Vs + kb * 32 * D, ko[ks]), df[ks], dp);
        if constexpr (D == 128) { if (ks % 2 == 1) __builtin_amdgcn_sched_barrier(0); }
      }
      mfma_prio(false);
      // S^T / dP^T: row = key k0 + (r&3)+8(r>>2)+4*h32, column = this lane's query
      const bool need_mask = (CAUSAL && (k0 + 31 > qw0 + off)) || (k0 + 32 > p.Tk);
      if (need_mask) {
        const int lim = vis - k0;
#pragma unroll
        for (int r = 0; r < 16; ++r)
          s[r] = ((r & 3) + 8 * (r >> 2) > lim) ? -INFINITY : s[r];
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pv = __builtin_amdgcn_exp2f(fmaf(s[r], c, -L));
        dp[r] = pv * (dp[r] - dl);  // dS^T / scale
      }
      const bf16x8 ds0 = acc_to_frag(dp, 0), ds1 = acc_to_frag(dp, 1);
      // dQ^T += K^T dS^T: A = K^T by transposed reads of the K image (key order permuted
      // within each 16-key step exactly as the accumulator-as-operand dS^T fragment)
      mfma_prio(true);
#pragma unroll
      for (int db = 0; db < NDB; ++db) {
        dq[db] = mfma32(tr_frag<D>(Ks, kb * 32 + 4 * h32, db * 32, lane, 8), ds0, dq[db]);
        dq[db] = mfma32(tr_frag<D>(Ks, kb * 32 + 16 + 4 * h32, db * 32, lane, 8), ds1, dq[db]);
      }
      mfma_prio(false);
    }
    if (t + 1 < ntiles) swrite(std::integral_constant<int, buf ^ 1>{});
    __syncthreads();
  };

  if (ntiles > 0) {
    gload(0);
    swrite(std::integral_constant<int, 0>{});
  }
  // retire the prologue loads with a wait the compiler can see (see attn_fwd_kernel)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  for (int t = 0; t < ntiles; t += 2) {
    tile(std::integral_constant<int, 0>{}, t);
    if (t + 1 < ntiles) tile(std::integral_constant<int, 1>{}, t + 1);
  }

  if (BIAS && qw0 < p.T)  // column sums of this wave's 32 queries (packed QKV bias grad)
    wave_colsum_store<NDB>(dq, p.scale, myq < p.T, l32, h32,
                           p.bias_part + ((long)b * ((p.T + 31) / 32) + qw0 / 32) * p.bias_ld + hq * D);
  if (myq < p.T) {
    ORION_DASSERT(b < p.B && hq < p.Hq);
    bf16_t* Qo = p.dq + b * p.dq_sb + hq * p.dq_sh + (long)myq * p.dq_st;
    const long rrow = (long)(myq + p.rope_pos0) * (D / 2);  // as the forward rope kernel (t + pos0)
    store_row_grad<NDB>(dq, p.scale, Qo, h32, p.rope_cos ? p.rope_cos + rrow : nullptr,
                        p.rope_sin ? p.rope_sin + rrow : nullptr);
  }
}

// ============================================================================ dQ, 4 waves/SIMD
// attn_bwd_dq4 (round 5, D = 64): the dQ kernel on attn_fwd4's recipe (csrc/attn_fwd.hip).
// The round-2..4 kernel above stages K / V through registers (gload / swrite) and leaves its
// LDS reads to the compiler: 150-156 VGPRs, three waves per SIMD.  Here K / V tiles arrive by
// LDS-DMA into a double buffer, every fragment read is inline asm at an immediate offset with
// a counted wait, and the chains run one after the other on shared fragment registers
// (S^T: K fragments; dP^T: V fragments; dQ^T: K^T halves), so the live set is Q and dO
// fragments 32, dQ 32, S / P 16, dP / dS 16 and one chain's fragments 16: under 128 VGPRs,
// four workgroups of 4 waves per CU (32 KB of LDS each).  Same numerics as attn_bwd_dq.
template <bool CAUSAL, bool BIAS>
__global__ __launch_bounds__(256, 4) void attn_bwd_dq4_kernel(AttnParams p) {
  constexpr int D = 64, BM = 128, BN = 64, TILE = BN * D, NDB = 2;
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];  // [2 bufs][K|V][TILE]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h32 = lane >> 5, l32 = lane & 31;
  const int BH = p.B * p.Hq;
  const int nqt = (p.T + BM - 1) / BM;
  const int bh = blockIdx.x % BH;
  const int qt = nqt - 1 - (int)(blockIdx.x / BH);  // heaviest (causal) tiles launch first
  const int b = bh / p.Hq, hq = bh % p.Hq, hk = hq / (p.Hq / p.Hkv);
  const int q0 = qt * BM, qw0 = q0 + wv * 32, myq = qw0 + l32;
  const int off = p.Tk - p.T;
  const float c = p.scale_log2;

  const bf16_t* Kb = p.k + b * p.k_sb + hk * p.k_sh;
  const bf16_t* Vb = p.v + b * p.v_sb + hk * p.v_sh;

  const int kend = CAUSAL ? min(p.Tk, q0 + BM + off) : p.Tk;
  const int ntiles = (kend + BN - 1) / BN;

  // LDS-DMA of K / V tiles as attn_fwd4_kernel: 8 pieces of 8 rows x 128 bytes per image, wave
  // wv issues pieces 2 wv, 2 wv + 1; the swizzle rides on the source chunk
  const unsigned kst_b = (unsigned)p.k_st * 2, vst_b = (unsigned)p.v_st * 2;
  const __amdgpu_buffer_rsrc_t rk = make_rsrc(Kb, (unsigned)((long)(p.Tk - 1) * p.k_st + D) * 2);
  const __amdgpu_buffer_rsrc_t rv = make_rsrc(Vb, (unsigned)((long)(p.Tk - 1) * p.v_st + D) * 2);
  const int prow0 = 16 * wv + (lane >> 3);
  auto dma = [&](int t, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    bf16_t* Ks = smem + buf * 2 * TILE;
    const int k0 = t * BN;
    // the per-lane source offsets are recomputed per call (opaque row): hoisted, the four of
    // them were spilled in the causal kernels
    int pr = prow0;
    asm volatile("" : "+v"(pr));
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int row = pr + 8 * e;
      const unsigned ch16 = 16u * (unsigned)((lane & 7) ^ swz<D>(row));
      if (k0 + BN <= p.Tk) {
        blds16(rk, (unsigned)row * kst_b + ch16, (unsigned)k0 * kst_b, Ks + (2 * wv + e) * 512);
        blds16(rv, (unsigned)row * vst_b + ch16, (unsigned)k0 * vst_b, Ks + TILE + (2 * wv + e) * 512);
      } else {  // last partial tile: rows past Tk re-read the last key (masked below)
        const unsigned key = (unsigned)min(k0 + row, p.Tk - 1);
        blds16(rk, key * kst_b + ch16, 0, Ks + (2 * wv + e) * 512);
        blds16(rv, key * vst_b + ch16, 0, Ks + TILE + (2 * wv + e) * 512);
      }
    }
  };
  // per-lane LDS byte bases: K / V rows l32 at d chunk 2 ks + h32 (the 32-key block by an
  // immediate); K^T transposed reads of key rows 4 h32 + (iq >> 2) (+ 8: second half), columns
  // db 32 + 16 (gq & 1) + 4 (iq & 3) (the 16-key step by an immediate: the swizzle does not
  // depend on it)
  // Registers are the budget here: one relative base per read family, the chunk index of
  // fragment ks / block db applied by an xor per read (loff's swizzle is an xor on the 16-byte
  // chunk: fragment ks is chunk (2 ks) ^ z, d block db flips chunk bit 2), kept opaque per
  // block so the compiler does not hoist the four addresses back into registers.
  const unsigned lds0 = lds_addr(smem, 0);
  const unsigned zk = 2u * (unsigned)loff<D>(l32, 8 * h32);  // fragment 0 (chunk h32 ^ swz)
  const int gq = lane >> 4, iq = lane & 15;
  unsigned ztr[2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf)
    ztr[hf] = 2u * (unsigned)loff<D>(4 * h32 + (iq >> 2) + 8 * hf, 16 * (gq & 1) + 4 * (iq & 3));
  // key k0 + rowoff(r) + 4 h32 of a 32-key block is visible to this lane's query iff
  // rowoff(r) <= vis - k0
  const int vis = (CAUSAL ? min(myq + off, p.Tk - 1) : p.Tk - 1) - 4 * h32;

  f32x16 dq[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db) dq[db] = zero16();

  // Prologue: the first K / V tile's DMA, then this wave's 32 query rows of Q, dO and O.
  // delta = rowsum(dO O) is computed here (the one kernel that owns each query row) and
  // written for the dK/dV kernel, which runs after this one -- no separate delta pass.  BIAS:
  // also the QKV bias gradient's K and V columns of this 32-token block (attn_delta_kernel's
  // identities: K columns 0, V columns the block's column sum of dO).
  if (ntiles > 0) dma(0, std::integral_constant<int, 0>{});
  bf16x8 qf[D / 16], df[D / 16];
  float L, dl;
  {
    const int qr = min(myq, p.T - 1);
    const bf16_t* Qr = p.q + b * p.q_sb + hq * p.q_sh + (long)qr * p.q_st;
    const bf16_t* Dr = p.dout + b * p.do_sb + hq * p.do_sh + (long)qr * p.do_st;
    const bf16_t* Or = p.o + b * p.o_sb + hq * p.o_sh + (long)qr * p.o_st;
    bf16x8 of[D / 16];
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      qf[ks] = *reinterpret_cast<const bf16x8*>(Qr + ks * 16 + 8 * h32);
      df[ks] = *reinterpret_cast<const bf16x8*>(Dr + ks * 16 + 8 * h32);
      of[ks] = *reinterpret_cast<const bf16x8*>(Or + ks * 16 + 8 * h32);
    }
    const long r = ((long)b * p.Hq + hq) * p.T + qr;
    L = p.lse[r];
    float d4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) d4[j & 3] = fmaf(bf2f(of[ks][j]), bf2f(df[ks][j]), d4[j & 3]);
    dl = (d4[0] + d4[1]) + (d4[2] + d4[3]);
    dl += __shfl_xor(dl, 32);  // the other d half of the row
    if (h32 == 0 && myq < p.T) const_cast<float*>(p.delta)[r] = dl;  // the scratch the dK/dV kernel reads
    if constexpr (BIAS) {
      if (qw0 < p.T) {  // T % 32 == 0: the wave's rows are one 32-token block
        float* prow = p.bias_part + ((long)b * (p.T / 32) + qw0 / 32) * p.bias_ld + (long)(p.Hq + hq) * D;
        float v[32];
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks)
#pragma unroll
          for (int j = 0; j < 8; ++j) v[8 * ks + j] = bf2f(df[ks][j]);
        wave_colsum_vals<32>(v, l32);
        // value index idx = l32 + ... -> column ks 16 + 8 h32 + j of idx = 8 ks + j
        const int d = (l32 >> 3) * 16 + 8 * h32 + (l32 & 7);
        prow[d] = 0.f;                    // K columns
        prow[(long)p.Hkv * D + d] = v[0];  // V columns
      }
    }
  }

  // one 32-key block (kb) of the tile in buffer BUF
  auto block = [&](int t, auto bufc, auto kbc) {
    constexpr int buf = decltype(bufc)::value, kb = decltype(kbc)::value;
    constexpr unsigned BOFF = buf * 2 * TILE * 2 + kb * 32 * D * 2;  // bytes: K block
    const int k0 = t * BN + kb * 32;
    if (CAUSAL && k0 > qw0 + 31 + off) return;  // wave-uniform: block fully masked
    f32x16 s = zero16(), dp = zero16();
    unsigned zb = zk, zt0 = ztr[0], zt1 = ztr[1];
    asm volatile("" : "+v"(zb), "+v"(zt0), "+v"(zt1));
    auto kad = [&](int ks) { return lds0 + (zb ^ (unsigned)(ks << 5)); };
    // S^T then dP^T on the same fragment registers
    auto chain = [&](f32x16& acc, const bf16x8 (&bop)[D / 16], auto offc) {
      constexpr unsigned O = decltype(offc)::value;
      // all four reads in flight; the MFMAs wait for them in order (reading two at a time
      // measured the same: 0.555-0.559 vs 0.554-0.558 ms)
      bf16x8 f[4];
      f[0] = b128_read_at<O>(kad(0));
      f[1] = b128_read_at<O>(kad(1));
      f[2] = b128_read_at<O>(kad(2));
      f[3] = b128_read_at<O>(kad(3));
      asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(f[0]), "+v"(f[1]));
      mfma_prio(true);
      acc = mfma32(f[0], bop[0], acc);
      acc = mfma32(f[1], bop[1], acc);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[2]), "+v"(f[3]));
      acc = mfma32(f[2], bop[2], acc);
      acc = mfma32(f[3], bop[3], acc);
      mfma_prio(false);
    };
    chain(s, qf, std::integral_constant<unsigned, BOFF>{});
    chain(dp, df, std::integral_constant<unsigned, BOFF + TILE * 2>{});
    // S^T / dP^T: row = key k0 + (r&3)+8(r>>2)+4*h32, column = this lane's query
    const bool need_mask = (CAUSAL && (k0 + 31 > qw0 + off)) || (k0 + 32 > p.Tk);
    if (need_mask) {
      const int lim = vis - k0;
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = ((r & 3) + 8 * (r >> 2) > lim) ? -INFINITY : s[r];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pv = __builtin_amdgcn_exp2f(fmaf(s[r], c, -L));
      dp[r] = pv * (dp[r] - dl);  // dS^T / scale
    }
    const bf16x8 ds0 = acc_to_frag(dp, 0), ds1 = acc_to_frag(dp, 1);
    // dQ^T += K^T dS^T: K^T by transposed reads, kept as halves until their wait
    constexpr unsigned T0 = buf * 2 * TILE * 2 + (2 * kb) * 16 * D * 2, T1 = T0 + 16 * D * 2;
    bf16x4 lo[NDB][2], hi[NDB][2];
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      const unsigned a0 = lds0 + (zt0 ^ (unsigned)(db << 6)), a1 = lds0 + (zt1 ^ (unsigned)(db << 6));
      lo[db][0] = tr_read_at<T0>(a0);
      hi[db][0] = tr_read_at<T0>(a1);
      lo[db][1] = tr_read_at<T1>(a0);
      hi[db][1] = tr_read_at<T1>(a1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(lo[0][0]), "+v"(lo[0][1]), "+v"(lo[1][0]), "+v"(lo[1][1]), "+v"(hi[0][0]),
                   "+v"(hi[0][1]), "+v"(hi[1][0]), "+v"(hi[1][1]));
    mfma_prio(true);
#pragma unroll
    for (int db = 0; db < NDB; ++db) {
      dq[db] = mfma32(cat8(lo[db][0], hi[db][0]), ds0, dq[db]);
      dq[db] = mfma32(cat8(lo[db][1], hi[db][1]), ds1, dq[db]);
    }
    mfma_prio(false);
  };
  auto tile = [&](int t, auto bufc) {
    constexpr int buf = decltype(bufc)::value;
    // tile t landed (this wave's pieces; the barrier: everyone's) and every wave is done with
    // the other buffer (read in tile t - 1): tile t + 1 may overwrite it
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < ntiles) dma(t + 1, std::integral_constant<int, buf ^ 1>{});
    block(t, bufc, std::integral_constant<int, 0>{});
    block(t, bufc, std::integral_constant<int, 1>{});
  };

  for (int t = 0; t < ntiles; t += 2) {
    tile(t, std::integral_constant<int, 0>{});
    if (t + 1 < ntiles) tile(t + 1, std::integral_constant<int, 1>{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA in flight when the workgroup ends

  if (BIAS && qw0 < p.T)  // column sums of this wave's 32 queries (packed QKV bias grad)
    wave_colsum_store<NDB>(dq, p.scale, myq < p.T, l32, h32,
                           p.bias_part + ((long)b * ((p.T + 31) / 32) + qw0 / 32) * p.bias_ld + hq * D);
  if (myq < p.T) {
    ORION_DASSERT(b < p.B && hq < p.Hq);
    bf16_t* Qo = p.dq + b * p.dq_sb + hq * p.dq_sh + (long)myq * p.dq_st;
    const long rrow = (long)(myq + p.rope_pos0) * (D / 2);
    store_row_grad<NDB>(dq, p.scale, Qo, h32, p.rope_cos ? p.rope_cos + rrow : nullptr,
                        p.rope_sin ? p.rope_sin + rrow : nullptr);
  }
}

}  // namespace orion

using namespace orion;

extern "C++" {

static size_t kv_lds(int D) {
  return (size_t)2 * 2 * 32 * D * 2 + 4 * 32 * 4 + (D == 128 ? (size_t)32 * 4 * D * 2 : 0);
}
static size_t dq_lds(int D) { return (size_t)2 * 2 * 64 * D * 2; }

template <int D, bool CAUSAL>
static void kv_launch(const AttnParams& q, int grid, hipStream_t st) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_kv_kernel<D, CAUSAL>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kv_lds(D));
    done = true;
  }
  attn_bwd_kv_kernel<D, CAUSAL><<<grid, kv_waves<D>() * 64, kv_lds(D), st>>>(q);
}

// ORION_ATTN_DQ=v3: the D = 64 dQ kernel of rounds 2-4 (A/B); default attn_bwd_dq4
static bool dq_v3() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ORION_ATTN_DQ");
    v = (e && strcmp(e, "v3") == 0) ? 1 : 0;
  }
  return v == 1;
}

template <bool CAUSAL, bool BIAS>
static void dq4_launch(const AttnParams& q, int grid, hipStream_t st) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_dq4_kernel<CAUSAL, BIAS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 2 * 64 * 64 * 2);
    done = true;
  }
  attn_bwd_dq4_kernel<CAUSAL, BIAS><<<grid, 256, 2 * 2 * 64 * 64 * 2, st>>>(q);
}

template <int D, bool CAUSAL, bool BIAS = false, bool FD = false>
static void dq_launch(const AttnParams& q, int grid, hipStream_t st) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_dq_kernel<D, CAUSAL, BIAS, FD>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)dq_lds(D));
    done = true;
  }
  attn_bwd_dq_kernel<D, CAUSAL, BIAS, FD><<<grid, 256, dq_lds(D), st>>>(q);
}

// ORION_ATTN_DELTA=pass: the separate delta pass at D = 128 (A/B); default: fused into dQ
static bool delta_pass() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ORION_ATTN_DELTA");
    v = (e && strcmp(e, "pass") == 0) ? 1 : 0;
  }
  return v == 1;
}

// delta (caller-allocated [B][Hq][T] fp32 scratch), dK/dV and dQ; p.dq / dk / dv are bf16
// outputs (strided views allowed).  Order on stream st: D = 64 -- dQ (attn_bwd_dq4, writes
// delta and the bias K / V columns), then dK/dV (reads delta); D = 128 -- dQ (attn_bwd_dq with
// the fused delta), then dK/dV; ORION_ATTN_DQ=v3 / ORION_ATTN_DELTA=pass -- the delta pass,
// dK/dV, dQ.
int orion_attn_bwd_split(const AttnParams& p, int D, bool causal, float* delta, hipStream_t st) {
  // 32-bit buffer offsets: the dQ kernel addresses one (batch, KV head)'s K / V, the dK/dV
  // kernel one batch's Q / dO over all query heads; beyond 2 GB the caller takes the fused
  // form (64-bit addressing)
  constexpr long LIM = 1L << 31;
  if (((long)(p.Tk - 1) * p.k_st + D) * 2 >= LIM || ((long)(p.Tk - 1) * p.v_st + D) * 2 >= LIM ||
      ((long)(p.T - 1) * p.q_st + (long)(p.Hq - 1) * p.q_sh + D) * 2 >= LIM ||
      ((long)(p.T - 1) * p.do_st + (long)(p.Hq - 1) * p.do_sh + D) * 2 >= LIM)
    return -2;
  const long rows = (long)p.B * p.Hq * p.T;
  const int pre_grid = (int)((rows * (D / 8) + 255) / 256);
  AttnParams q = p;
  q.delta = delta;
  const int kv_grid = ((p.Tk + 32 * 4 - 1) / (32 * 4)) * p.B * p.Hkv;
  const int dq_grid = ((p.T + 127) / 128) * p.B * p.Hq;
  static const bool diag = getenv("ORION_ATTN_DIAG") && getenv("ORION_ATTN_DIAG")[0] == '1';
  if (diag && D == 64) {  // stamped dK/dV kernel only, stamps over p.dq (scripts/attn_stamps.py)
    attn_delta_kernel<64><<<pre_grid, 256, 0, st>>>(p, delta);
    if (causal) {
      (void)hipFuncSetAttribute((const void*)attn_bwd_kv_kernel<64, true, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kv_lds(64));
      attn_bwd_kv_kernel<64, true, true><<<kv_grid, kv_waves<64>() * 64, kv_lds(64), st>>>(q);
    } else {
      (void)hipFuncSetAttribute((const void*)attn_bwd_kv_kernel<64, false, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)kv_lds(64));
      attn_bwd_kv_kernel<64, false, true><<<kv_grid, kv_waves<64>() * 64, kv_lds(64), st>>>(q);
    }
    return (int)hipGetLastError();
  }
  // D = 64 (attn_bwd_dq4): the dQ kernel first -- it computes delta (and, with the QKV bias,
  // the K / V bias columns) in its prologue -- then dK/dV, which reads delta.  Otherwise (and
  // with ORION_ATTN_DQ=v3): the delta pass, dK/dV, dQ.
  const bool dq4 = D == 64 && !dq_v3();
  if (p.bias_part) {  // packed self-attention with the QKV bias gradient (GPT-2: D = 64, MHA)
    if (D != 64 || p.T != p.Tk || p.Hq != p.Hkv || p.T % 32) return -3;
    if (dq4) {
      if (causal) {
        dq4_launch<true, true>(q, dq_grid, st);
        kv_launch<64, true>(q, kv_grid, st);
      } else {
        dq4_launch<false, true>(q, dq_grid, st);
        kv_launch<64, false>(q, kv_grid, st);
      }
      return (int)hipGetLastError();
    }
#define SPLITB(CC)                                                                                  \
  attn_delta_kernel<64, true><<<pre_grid, 256, 0, st>>>(q, delta);                                  \
  kv_launch<64, CC>(q, kv_grid, st);                                                                \
  dq_launch<64, CC, true>(q, dq_grid, st);
    if (causal) { SPLITB(true) } else { SPLITB(false) }
#undef SPLITB
    return (int)hipGetLastError();
  }
  if (dq4) {
    if (causal) {
      dq4_launch<true, false>(q, dq_grid, st);
      kv_launch<64, true>(q, kv_grid, st);
    } else {
      dq4_launch<false, false>(q, dq_grid, st);
      kv_launch<64, false>(q, kv_grid, st);
    }
    return (int)hipGetLastError();
  }
#define SPLIT(DD, CC)                                    \
  attn_delta_kernel<DD><<<pre_grid, 256, 0, st>>>(p, delta); \
  kv_launch<DD, CC>(q, kv_grid, st);                       \
  dq_launch<DD, CC>(q, dq_grid, st);
  if (D == 64) {
    if (causal) { SPLIT(64, true) } else { SPLIT(64, false) }
  } else if (D == 128 && !delta_pass()) {  // dQ first: it writes delta for dK/dV
    if (causal) {
      dq_launch<128, true, false, true>(q, dq_grid, st);
      kv_launch<128, true>(q, kv_grid, st);
    } else {
      dq_launch<128, false, false, true>(q, dq_grid, st);
      kv_launch<128, false>(q, kv_grid, st);
    }
  } else if (D == 128) {
    if (causal) { SPLIT(128, true) } else { SPLIT(128, false) }
  } else {
    return -1;
  }
#undef SPLIT
  return (int)hipGetLastError();
}

}  // extern "C++"
