// LayerNorm forward / backward for bf16 activations (K3 in SURVEY.md §2.11).
//
// Regime: memory bound (one read of x, one write of y; bwd reads x, dy, writes dx).
// Design for wave64:
//   * one wavefront per row, 4 rows per 256-thread workgroup; a lane owns the
//     same VEC-wide column slices in every row it touches, so its slice of
//     gamma/beta lives in registers and the backward's column sums
//     (dgamma, dbeta) accumulate in registers with no atomics;
//   * row statistics by 64-lane butterfly (__shfl_xor), two-pass variance in
//     registers (the row is read from HBM once);
//   * backward: a fixed grid of row-chunk workgroups writes fp32 partial column
//     sums, a second tiny kernel folds them (deterministic, no float atomics).
#include <cstdlib>

#include "common.h"

// LN_NT: the residual stream sum (saved for the backward, read again by the next block's norm
// several kernels later) is stored, and the far operands (the incoming residual; the saved
// input in the backward) are loaded, with the non-temporal hint, so the caches keep what the
// NEXT kernel reads (the normalised output, the incoming gradient).
#ifndef LN_NT
#define LN_NT 1  // GPT-2 step: LayerNorm backward 78.5 vs 83.1 us, the GEMMs after it 1-2 % (profiles/ab/ln_nt_r04.log)
#endif

#ifndef LN_DRES_NT
#define LN_DRES_NT 1  // the incoming residual gradient (written several kernels earlier): LN bwd 77.9 vs 79.1 us (profiles/ab/ln_dres_nt_r04.log)
#endif

namespace orion {

template <typename T>
ORION_DEVICE T ld_far(const T* p) {
  if constexpr (LN_NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <int VEC>
ORION_DEVICE void store_vec_far(bf16_t* p, const float* in) {
  typedef typename VecT<VEC>::type V;
  V v;
#pragma unroll
  for (int j = 0; j < VEC; ++j) v[j] = f2bf(in[j]);
  if constexpr (LN_NT) __builtin_nontemporal_store(v, reinterpret_cast<V*>(p));
  else *reinterpret_cast<V*>(p) = v;
}

template <int VEC>
ORION_DEVICE void load_vec(const bf16_t* p, float* out) {
  typedef typename VecT<VEC>::type V;
  V v = *reinterpret_cast<const V*>(p);
#pragma unroll
  for (int j = 0; j < VEC; ++j) out[j] = bf2f(v[j]);
}

template <int VEC>
ORION_DEVICE void store_vec(bf16_t* p, const float* in) {
  typedef typename VecT<VEC>::type V;
  V v;
#pragma unroll
  for (int j = 0; j < VEC; ++j) v[j] = f2bf(in[j]);
  *reinterpret_cast<V*>(p) = v;
}

template <int VEC, int ITERS>
__global__ __launch_bounds__(256) void ln_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
    bf16_t* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out,
    int rows, int C, float eps, const bf16_t* __restrict__ res, bf16_t* __restrict__ sum_out,
    const bf16_t* __restrict__ rbias, const int64_t* __restrict__ idx, int T, long V, int* err) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  // idx: embedding gather -- x is the token table (row idx[row]) and res the position table
  // (row row % T), so s = wte[idx] + wpe[t] is formed, returned and normalised in one pass.
  // An id outside [0, V) never addresses memory: it reads table row 0 and raises the error
  // flag (ops/embedding.py reports it).
  long id = row;
  if (idx) {
    id = idx[row];
    ORION_DASSERT(id >= 0 && id < V);
    if ((unsigned long)id >= (unsigned long)V) {
      if (lane == 0) atomicOr(err, 1);
      id = 0;
    }
  }
  const bf16_t* xr = x + (size_t)id * C;
  const size_t rrow = idx ? (size_t)(row % T) : (size_t)row;
  // Every load of the row (x, residual, branch bias, gamma, beta) is issued, unconditionally
  // and as raw bf16 vectors, before the first store: on CDNA4 vmcnt counts stores, so a load
  // after the sum store would wait for it, and per-operand branches (or conversions right
  // after each load) made the compiler wait for every load in turn.  Absent operands read a
  // stand-in row, columns past C the last chunk (their results are not stored).
  typedef typename VecT<VEC>::type VT;
  const bf16_t* rp = res ? res + rrow * C : xr;
  const bf16_t* rbp = (res && rbias) ? rbias : w;
  const bf16_t* bp = b ? b : w;
  VT xv[ITERS], rvv[ITERS], rbv[ITERS], wv[ITERS], bvv[ITERS];
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int cl = min((i * 64 + lane) * VEC, C - VEC);
    xv[i] = *reinterpret_cast<const VT*>(xr + cl);
    rvv[i] = ld_far(reinterpret_cast<const VT*>(rp + cl));
    rbv[i] = *reinterpret_cast<const VT*>(rbp + cl);
    wv[i] = *reinterpret_cast<const VT*>(w + cl);
    bvv[i] = *reinterpret_cast<const VT*>(bp + cl);
  }
  float v[ITERS][VEC];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int c = (i * 64 + lane) * VEC;
    if (c < C) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[i][j] = bf2f(xv[i][j]);
      if (res) {  // fused residual add: s = x + r is both returned and normalised
        float rv[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) rv[j] = bf2f(rvv[i][j]);
        if (rbias) {  // the branch's output-projection bias, added here instead of in the GEMM
#pragma unroll
          for (int j = 0; j < VEC; ++j) rv[j] = bf2f(f2bf(rv[j] + bf2f(rbv[i][j])));
        }
#pragma unroll
        for (int j = 0; j < VEC; ++j) v[i][j] = bf2f(f2bf(v[i][j] + rv[j]));
        store_vec_far<VEC>(sum_out + (size_t)row * C + c, v[i]);
      }
#pragma unroll
      for (int j = 0; j < VEC; ++j) s += v[i][j];
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[i][j] = 0.f;
    }
  }
  const float invC = 1.f / (float)C;
  const float mean = wave_sum(s) * invC;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int c = (i * 64 + lane) * VEC;
    if (c < C) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) * invC + eps);
  bf16_t* yr = y + (size_t)row * C;
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int c = (i * 64 + lane) * VEC;
    if (c < C) {
      float o[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = (v[i][j] - mean) * rstd * bf2f(wv[i][j]) + (b ? bf2f(bvv[i][j]) : 0.f);
      store_vec<VEC>(yr + c, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Single-input forward (round 6: the residual sites' LayerNorm reads only the new stream, the
// branch GEMM having done the add).  gamma / beta stay in registers for the wave's whole row
// list (the per-row kernel above reloads them, and stand-ins for the absent operands, for every
// row), and the next row's loads are issued before this row's stores (two register sets), so a
// wave keeps two rows in flight.
template <int VEC, int ITERS>
__global__ __launch_bounds__(256) void ln_fwd1_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                      const bf16_t* __restrict__ b, bf16_t* __restrict__ y,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                      int rows, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
  typedef typename VecT<VEC>::type VT;
  float wf[ITERS][VEC], bf[ITERS][VEC];
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int cl = min((i * 64 + lane) * VEC, C - VEC);
    load_vec<VEC>(w + cl, wf[i]);
    if (b) load_vec<VEC>(b + cl, bf[i]);
    else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) bf[i][j] = 0.f;
    }
  }
  const float invC = 1.f / (float)C;
  auto load = [&](int r, VT (&v)[ITERS]) {
    if (r >= rows) return;  // wave-uniform
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const int cl = min((i * 64 + lane) * VEC, C - VEC);
      v[i] = *reinterpret_cast<const VT*>(x + (size_t)r * C + cl);
    }
  };
  auto proc = [&](int r, const VT (&v)[ITERS]) {
    float f[ITERS][VEC];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const bool ok = (i * 64 + lane) * VEC < C;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        f[i][j] = ok ? bf2f(v[i][j]) : 0.f;
        s += f[i][j];
      }
    }
    const float mean = wave_sum(s) * invC;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const bool ok = (i * 64 + lane) * VEC < C;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float d = ok ? f[i][j] - mean : 0.f;
        q += d * d;
      }
    }
    const float rstd = rsqrtf(wave_sum(q) * invC + eps);
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const int c = (i * 64 + lane) * VEC;
      if (c < C) {
        float o[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) o[j] = (f[i][j] - mean) * rstd * wf[i][j] + bf[i][j];
        store_vec<VEC>(y + (size_t)r * C + c, o);
      }
    }
    if (lane == 0) {
      mean_out[r] = mean;
      rstd_out[r] = rstd;
    }
  };
  VT va[ITERS], vb[ITERS];
  int r = wid;
  load(r, va);
  for (; r < rows; r += 2 * nw) {
    load(r + nw, vb);
    proc(r, va);
    if (r + nw >= rows) break;
    load(r + 2 * nw, va);
    proc(r + nw, vb);
  }
}

// Backward: dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * gamma.
template <int VEC, int ITERS, bool EXACT = false>  // EXACT: ITERS * 64 * VEC == C (no column guards)
__global__ __launch_bounds__(256) void ln_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    bf16_t* __restrict__ dx, float* __restrict__ part_dw, float* __restrict__ part_db,
    int rows, int C, int rows_per_block, const bf16_t* __restrict__ dres,
    float* __restrict__ part_dx) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4][C]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float wf[ITERS][VEC], adw[ITERS][VEC], adb[ITERS][VEC], adx[ITERS][VEC];
#pragma unroll
  for (int i = 0; i < ITERS; ++i) {
    const int c = (i * 64 + lane) * VEC;
    if (c < C) load_vec<VEC>(w + c, wf[i]);
    else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) wf[i][j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) { adw[i][j] = 0.f; adb[i][j] = 0.f; adx[i][j] = 0.f; }
  }
  const float invC = 1.f / (float)C;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  typedef typename VecT<VEC>::type V;
  // One row per wave per step, software-pipelined over two register sets: the loads of the
  // wave's next row are issued BEFORE this row's dx stores.  On CDNA4 vmcnt counts stores
  // too, so a load issued after a store is waited for behind that store's completion; with
  // the loads of row r + 4 ahead of the stores of row r, the wait for them leaves the
  // stores in flight (the two-rows-then-stores form serialised every step on its stores).
  auto load_row = [&](int rw, V (&xr)[ITERS], V (&dyr)[ITERS], V (&rr)[ITERS]) {
    if (rw >= r1) return;  // wave-uniform
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const int c = (i * 64 + lane) * VEC;
      if (EXACT || c < C) {
        xr[i] = ld_far(reinterpret_cast<const V*>(x + (size_t)rw * C + c));
        dyr[i] = *reinterpret_cast<const V*>(dy + (size_t)rw * C + c);
        if (dres) {
          if constexpr (LN_DRES_NT) rr[i] = ld_far(reinterpret_cast<const V*>(dres + (size_t)rw * C + c));
          else rr[i] = *reinterpret_cast<const V*>(dres + (size_t)rw * C + c);
        }
      }
    }
  };
  auto proc_row = [&](int rw, const V (&xr)[ITERS], const V (&dyr)[ITERS], const V (&rr)[ITERS]) {
    const float mean = mean_in[rw], rstd = rstd_in[rw];
    float xh[ITERS][VEC], g[ITERS][VEC];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const int c = (i * 64 + lane) * VEC;
      if (EXACT || c < C) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float dv = bf2f(dyr[i][j]);
          xh[i][j] = (bf2f(xr[i][j]) - mean) * rstd;
          g[i][j] = dv * wf[i][j];
          s1 += g[i][j];
          s2 += g[i][j] * xh[i][j];
          adw[i][j] += dv * xh[i][j];
          adb[i][j] += dv;
        }
      } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) { xh[i][j] = 0.f; g[i][j] = 0.f; }
      }
    }
    const float m1 = wave_sum(s1) * invC, m2 = wave_sum(s2) * invC;
    bf16_t* dxr = dx + (size_t)rw * C;
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const int c = (i * 64 + lane) * VEC;
      if (EXACT || c < C) {
        float o[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          o[j] = rstd * (g[i][j] - m1 - xh[i][j] * m2);
          if (dres) o[j] += bf2f(rr[i][j]);  // gradient arriving through the residual stream
        }
        if (part_dx) {
#pragma unroll
          for (int j = 0; j < VEC; ++j) adx[i][j] += bf2f(f2bf(o[j]));
        }
        store_vec<VEC>(dxr + c, o);
      }
    }
  };
  V xa[ITERS], da[ITERS], ra[ITERS], xb[ITERS], db[ITERS], rb[ITERS];
  int row = r0 + wv;
  load_row(row, xa, da, ra);
  for (; row < r1; row += 8) {
    load_row(row + 4, xb, db, rb);
    proc_row(row, xa, da, ra);
    if (row + 4 >= r1) break;
    load_row(row + 8, xa, da, ra);
    proc_row(row + 4, xb, db, rb);
  }
  // fold the 4 waves' column partials through LDS, one output pass per quantity
  if (part_dw) {
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const int c = (i * 64 + lane) * VEC;
      if (c < C) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) red[wv * C + c + j] = adw[i][j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256)
      part_dw[(size_t)blockIdx.x * C + c] = red[c] + red[C + c] + red[2 * C + c] + red[3 * C + c];
    __syncthreads();
  }
  if (part_db) {
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const int c = (i * 64 + lane) * VEC;
      if (c < C) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) red[wv * C + c + j] = adb[i][j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256)
      part_db[(size_t)blockIdx.x * C + c] = red[c] + red[C + c] + red[2 * C + c] + red[3 * C + c];
    __syncthreads();
  }
  if (part_dx) {
#pragma unroll
    for (int i = 0; i < ITERS; ++i) {
      const int c = (i * 64 + lane) * VEC;
      if (c < C) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) red[wv * C + c + j] = adx[i][j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256)
      part_dx[(size_t)blockIdx.x * C + c] = red[c] + red[C + c] + red[2 * C + c] + red[3 * C + c];
  }
}

// Two-stage column sum of fp32 partials part[P][C] -> bf16 out[C].
// Stage 1: grid (ceil(C/64), S); workgroup (s, cblk) folds rows [s*P/S, (s+1)*P/S) of 64
// columns with 4 waves x 8 independent loads in flight per lane (latency-bound otherwise).
__global__ __launch_bounds__(256) void colsum_stage1_kernel(const float* __restrict__ part,
                                                            float* __restrict__ mid, int P, int C,
                                                            int rows_per_split) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int p0 = blockIdx.y * rows_per_split, p1 = min(P, p0 + rows_per_split);
  float s = 0.f;
  if (c < C) {
    int p = p0 + wv;
    for (; p + 28 < p1; p += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(p + 4 * u) * C + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; p < p1; p += 4) s += part[(size_t)p * C + c];
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && c < C) mid[(size_t)blockIdx.y * C + c] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

__global__ __launch_bounds__(256) void colsum_stage2_kernel(const float* __restrict__ mid,
                                                            void* __restrict__ out, int S, int C,
                                                            int f32) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int i = 0; i < S; ++i) s += mid[(size_t)i * C + c];
  store_grad(out, c, s, f32);
}

constexpr int COLSUM_SPLITS = 16;

// The LN backward's three column sums (dgamma, dbeta, branch-bias grad) in one launch
// pair: blockIdx.z picks the [P][C] partial matrix part + z*P*C; z whose output is
// null is skipped (block-uniform exit, before any barrier).
struct ColsumOuts {
  void* out[3];
  int f32;  // outputs are fp32 (gradient arena) rather than bf16
};

__global__ __launch_bounds__(256) void colsum3_stage1_kernel(const float* __restrict__ part,
                                                             float* __restrict__ mid, int P, int C,
                                                             int rows_per_split, ColsumOuts o) {
  if (!o.out[blockIdx.z]) return;
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const float* pz = part + (size_t)blockIdx.z * P * C;
  const int p0 = blockIdx.y * rows_per_split, p1 = min(P, p0 + rows_per_split);
  float s = 0.f;
  if (c < C) {
    int p = p0 + wv;
    for (; p + 28 < p1; p += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = pz[(size_t)(p + 4 * u) * C + c];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; p < p1; p += 4) s += pz[(size_t)p * C + c];
  }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && c < C)
    mid[((size_t)blockIdx.z * gridDim.y + blockIdx.y) * C + c] =
        red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

__global__ __launch_bounds__(256) void colsum3_stage2_kernel(const float* __restrict__ mid, int S,
                                                             int C, ColsumOuts o) {
  void* out = o.out[blockIdx.y];
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (!out || c >= C) return;
  const float* mz = mid + (size_t)blockIdx.y * S * C;
  float s = 0.f;
  for (int i = 0; i < S; ++i) s += mz[(size_t)i * C + c];
  store_grad(out, c, s, o.f32);
}

// One-pass form (round 6, the default): workgroup (column block, z) folds ALL P rows of its
// CW columns -- lane = (row 64 / CW sub-row, column), NW waves, wave w rows (w + NW k) 64 / CW +
// sub with 16 loads in flight per lane, then the NW x 64 / CW partial sums in a fixed order --
// so the two ~5 us launches of the two-stage form become one (the partials were just written:
// they are read from the caches).  Narrow column blocks give the launch enough workgroups
// (C = 768: 48 per output).  Deterministic.
template <int NW, int CW>
__global__ __launch_bounds__(NW * 64) void colsum_onepass_kernel(const float* __restrict__ part, long zstride,
                                                                 int P, int C, ColsumOuts o) {
  constexpr int R = 64 / CW;  // rows per wave load
  void* out = o.out[blockIdx.y];
  if (!out) return;  // block-uniform, before the barrier
  __shared__ float red[NW * R][CW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int sub = lane / CW, cl = lane % CW;
  const int c = blockIdx.x * CW + cl;
  const float* pz = part + blockIdx.y * zstride;
  float s = 0.f;
  if (c < C) {
    // 16 predicated loads in flight per lane: P <= 1024 rows is ONE round trip per lane
    constexpr int STEP = NW * R, U = 16;
    for (int p = wv * R + sub; p < P; p += U * STEP) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = p + u * STEP < P ? pz[(size_t)(p + u * STEP) * C + c] : 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) s += v[u];
    }
  }
  red[wv * R + sub][cl] = s;
  __syncthreads();
  if (threadIdx.x < CW && c < C) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NW * R; ++w) t += red[w][cl];
    store_grad(out, c, t, o.f32);
  }
}

}  // namespace orion

using namespace orion;

int orion_colsum_partials2(const float* part, float* mid, void* out, int P, int C, int f32,
                           hipStream_t st);

// ORION_COLSUM=2: the two-stage column sums (A/B); default one pass
static bool colsum_two_stage() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ORION_COLSUM");
    v = (e && e[0] == '2') ? 1 : 0;
  }
  return v == 1;
}
constexpr int COLSUM_NW = 16, COLSUM_CW = 16;

// exact_fit: 4-wide slices when they tile the row exactly and 8-wide ones would not
// (C = 768: 3 x 64 x 4 uses every lane, 2 x 64 x 8 leaves a third idle).  Measured on
// MI355X at 65536 x 768: the backward gains from it, the forward does not (its 16-byte
// loads win), so only the backward asks for it.
static bool ln_pick(int C, int* vec, int* iters, bool exact_fit = false) {
  if (exact_fit && C % 256 == 0 && C % 512 != 0 && C <= 1024) {
    *vec = 4;
    *iters = C / 256;
  } else if (C % 8 == 0) {
    *vec = 8;
    *iters = (C + 511) / 512;
  } else if (C % 4 == 0) {
    *vec = 4;
    *iters = (C + 255) / 256;
  } else {
    return false;
  }
  return *iters <= 4;
}

int orion_ln_max_cols() { return 2048; }

// ORION_LN_FWD1=0: the single-input forward through the per-row kernel (A/B);
// ORION_LN_FWD1_BLOCKS: its workgroup count (default 4096: 4 rows per wave at 65,536 rows;
// 65,536 x 768: 256 / 512 / 1,024 / 2,048 / 4,096 blocks 67.0 / 41.6 / 36.4 / 36.7 / 35.8 us against
// 38.9 us for the per-row kernel)
static int ln_fwd1_blocks() {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("ORION_LN_FWD1");
    const char* nb = getenv("ORION_LN_FWD1_BLOCKS");
    v = (e && e[0] == '0') ? 0 : (nb ? atoi(nb) : 4096);
  }
  return v;
}

int orion_layernorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean,
                        float* rstd, int rows, int C, float eps, const void* res, void* sum_out,
                        const void* rbias, hipStream_t st, const int64_t* idx, int T, long V,
                        int* err) {
  int vec, it;
  if (!ln_pick(C, &vec, &it)) return -1;
  const int nb1 = ln_fwd1_blocks();
  if (!res && !idx && !rbias && !sum_out && nb1 > 0) {
    const int blocks = min(nb1, (rows + 3) / 4);
    auto X = (const bf16_t*)x; auto W = (const bf16_t*)w; auto B = (const bf16_t*)b; auto Y = (bf16_t*)y;
#define LNF1(VV, II) ln_fwd1_kernel<VV, II><<<blocks, 256, 0, st>>>(X, W, B, Y, mean, rstd, rows, C, eps)
    if (vec == 8) {
      switch (it) { case 1: LNF1(8, 1); break; case 2: LNF1(8, 2); break; case 3: LNF1(8, 3); break; default: LNF1(8, 4); }
    } else {
      switch (it) { case 1: LNF1(4, 1); break; case 2: LNF1(4, 2); break; case 3: LNF1(4, 3); break; default: LNF1(4, 4); }
    }
#undef LNF1
    return (int)hipGetLastError();
  }
  dim3 grid((rows + 3) / 4), block(256);
  auto X = (const bf16_t*)x; auto W = (const bf16_t*)w; auto B = (const bf16_t*)b;
  auto Y = (bf16_t*)y;
  auto R = (const bf16_t*)res; auto S = (bf16_t*)sum_out; auto RB = (const bf16_t*)rbias;
  if (vec == 8) {
    switch (it) {
      case 1: ln_fwd_kernel<8, 1><<<grid, block, 0, st>>>(X, W, B, Y, mean, rstd, rows, C, eps, R, S, RB, idx, T, V, err); break;
      case 2: ln_fwd_kernel<8, 2><<<grid, block, 0, st>>>(X, W, B, Y, mean, rstd, rows, C, eps, R, S, RB, idx, T, V, err); break;
      case 3: ln_fwd_kernel<8, 3><<<grid, block, 0, st>>>(X, W, B, Y, mean, rstd, rows, C, eps, R, S, RB, idx, T, V, err); break;
      case 4: ln_fwd_kernel<8, 4><<<grid, block, 0, st>>>(X, W, B, Y, mean, rstd, rows, C, eps, R, S, RB, idx, T, V, err); break;
    }
  } else {
    switch (it) {
      case 1: ln_fwd_kernel<4, 1><<<grid, block, 0, st>>>(X, W, B, Y, mean, rstd, rows, C, eps, R, S, RB, idx, T, V, err); break;
      case 2: ln_fwd_kernel<4, 2><<<grid, block, 0, st>>>(X, W, B, Y, mean, rstd, rows, C, eps, R, S, RB, idx, T, V, err); break;
      case 3: ln_fwd_kernel<4, 3><<<grid, block, 0, st>>>(X, W, B, Y, mean, rstd, rows, C, eps, R, S, RB, idx, T, V, err); break;
      case 4: ln_fwd_kernel<4, 4><<<grid, block, 0, st>>>(X, W, B, Y, mean, rstd, rows, C, eps, R, S, RB, idx, T, V, err); break;
    }
  }
  return (int)hipGetLastError();
}

// Number of row-chunk workgroups the backward uses (caller sizes the partial buffers).
int orion_layernorm_bwd_blocks(int rows) {
  int nb = (rows + 63) / 64;  // >= 64 rows (16 per wave) per workgroup
  return nb < 1024 ? (nb < 1 ? 1 : nb) : 1024;
}

template <int VEC, int ITERS>
static int ln_bwd_resident(size_t lds) {
  static int per_cu = 0;
  if (!per_cu) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, ln_bwd_kernel<VEC, ITERS>, 256, lds) != hipSuccess || n < 1)
      n = 1;
    per_cu = n;
  }
  return per_cu;
}

static int ln_bwd_grid(int rows, int vec, int it, size_t lds) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  }
  int per_cu = 1;
  if (vec == 8) {
    switch (it) {
      case 1: per_cu = ln_bwd_resident<8, 1>(lds); break;
      case 2: per_cu = ln_bwd_resident<8, 2>(lds); break;
      case 3: per_cu = ln_bwd_resident<8, 3>(lds); break;
      default: per_cu = ln_bwd_resident<8, 4>(lds); break;
    }
  } else {
    switch (it) {
      case 1: per_cu = ln_bwd_resident<4, 1>(lds); break;
      case 2: per_cu = ln_bwd_resident<4, 2>(lds); break;
      case 3: per_cu = ln_bwd_resident<4, 3>(lds); break;
      default: per_cu = ln_bwd_resident<4, 4>(lds); break;
    }
  }
  const int cap = orion_layernorm_bwd_blocks(rows);
  const int one_round = per_cu * cus;
  return one_round < cap ? one_round : cap;
}

int orion_layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean,
                        const float* rstd, void* dx, void* dw, void* db, float* part, int rows,
                        int C, const void* dres, void* drbias, int grad_f32, hipStream_t st) {
  int vec, it;
  if (!ln_pick(C, &vec, &it, /*exact_fit=*/true)) return -1;
  // One resident round of workgroups: the kernel strides over its rows, so a grid larger
  // than what fits at once leaves a partial second round (at 152 VGPRs three 4-wave
  // workgroups fit per CU: 1024 workgroups ran as 768 + 256).  The scratch is sized for
  // orion_layernorm_bwd_blocks(rows) >= nb.
  const int nb = ln_bwd_grid(rows, vec, it, (size_t)4 * C * sizeof(float));
  const int rpb = (rows + nb - 1) / nb;
  float* pdw = dw ? part : nullptr;
  float* pdb = db ? part + (size_t)nb * C : nullptr;
  float* pdx = drbias ? part + 2 * (size_t)nb * C : nullptr;
  const size_t lds = (size_t)4 * C * sizeof(float);
  auto DY = (const bf16_t*)dy; auto X = (const bf16_t*)x; auto W = (const bf16_t*)w;
  auto DX = (bf16_t*)dx;
  auto DR = (const bf16_t*)dres;
  if (vec == 8) {
    switch (it) {
      case 1: ln_bwd_kernel<8, 1><<<nb, 256, lds, st>>>(DY, X, W, mean, rstd, DX, pdw, pdb, rows, C, rpb, DR, pdx); break;
      case 2: ln_bwd_kernel<8, 2><<<nb, 256, lds, st>>>(DY, X, W, mean, rstd, DX, pdw, pdb, rows, C, rpb, DR, pdx); break;
      case 3: ln_bwd_kernel<8, 3><<<nb, 256, lds, st>>>(DY, X, W, mean, rstd, DX, pdw, pdb, rows, C, rpb, DR, pdx); break;
      case 4: ln_bwd_kernel<8, 4><<<nb, 256, lds, st>>>(DY, X, W, mean, rstd, DX, pdw, pdb, rows, C, rpb, DR, pdx); break;
    }
  } else if (C == it * 256) {  // exact fit (GPT-2: C = 768): no column guards
    switch (it) {
      case 1: ln_bwd_kernel<4, 1, true><<<nb, 256, lds, st>>>(DY, X, W, mean, rstd, DX, pdw, pdb, rows, C, rpb, DR, pdx); break;
      case 2: ln_bwd_kernel<4, 2, true><<<nb, 256, lds, st>>>(DY, X, W, mean, rstd, DX, pdw, pdb, rows, C, rpb, DR, pdx); break;
      case 3: ln_bwd_kernel<4, 3, true><<<nb, 256, lds, st>>>(DY, X, W, mean, rstd, DX, pdw, pdb, rows, C, rpb, DR, pdx); break;
      case 4: ln_bwd_kernel<4, 4, true><<<nb, 256, lds, st>>>(DY, X, W, mean, rstd, DX, pdw, pdb, rows, C, rpb, DR, pdx); break;
    }
  } else {
    switch (it) {
      case 1: ln_bwd_kernel<4, 1><<<nb, 256, lds, st>>>(DY, X, W, mean, rstd, DX, pdw, pdb, rows, C, rpb, DR, pdx); break;
      case 2: ln_bwd_kernel<4, 2><<<nb, 256, lds, st>>>(DY, X, W, mean, rstd, DX, pdw, pdb, rows, C, rpb, DR, pdx); break;
      case 3: ln_bwd_kernel<4, 3><<<nb, 256, lds, st>>>(DY, X, W, mean, rstd, DX, pdw, pdb, rows, C, rpb, DR, pdx); break;
      case 4: ln_bwd_kernel<4, 4><<<nb, 256, lds, st>>>(DY, X, W, mean, rstd, DX, pdw, pdb, rows, C, rpb, DR, pdx); break;
    }
  }
  float* mid = part + 3 * (size_t)nb * C;
  if (dw || db || drbias) {
    const ColsumOuts o{{dw, db, drbias}, grad_f32};
    if (!colsum_two_stage()) {
      colsum_onepass_kernel<COLSUM_NW, COLSUM_CW><<<dim3((C + COLSUM_CW - 1) / COLSUM_CW, 3), COLSUM_NW * 64, 0, st>>>(part, (long)nb * C, nb, C, o);
    } else {
      const int rps = (nb + COLSUM_SPLITS - 1) / COLSUM_SPLITS;
      colsum3_stage1_kernel<<<dim3((C + 63) / 64, COLSUM_SPLITS, 3), 256, 0, st>>>(part, mid, nb, C, rps, o);
      colsum3_stage2_kernel<<<dim3((C + 255) / 256, 3), 256, 0, st>>>(mid, COLSUM_SPLITS, C, o);
    }
  }
  return (int)hipGetLastError();
}

// Column sum of a bf16 matrix [rows][C] into bf16 out[C] (bias gradients); uses the
// same partial scheme.  part must hold orion_layernorm_bwd_blocks(rows) * C floats.
__global__ __launch_bounds__(256) void colsum_bf16_partial_kernel(
    const bf16_t* __restrict__ m, float* __restrict__ part, int rows, int C, int rows_per_block) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = (blockIdx.y * 64 + lane) * 8;
  const bool valid = c < C;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int r0 = blockIdx.x * rows_per_block, r1 = valid ? min(rows, r0 + rows_per_block) : 0;
  for (int r = r0 + wv; r < r1; r += 4) {
    float v[8];
    load_vec<8>(m + (size_t)r * C + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
  __shared__ float red[4][512];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[wv][lane * 8 + j] = acc[j];
  __syncthreads();
  if (wv == 0 && valid) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = lane * 8 + j;
      part[(size_t)blockIdx.x * C + c + j] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
    }
  }
}

int orion_colsum_bf16(const void* m, void* out, float* part, int rows, int C, int out_f32,
                      hipStream_t st) {
  if (C % 8) return -1;
  const int nb = orion_layernorm_bwd_blocks(rows);
  const int rpb = (rows + nb - 1) / nb;
  dim3 grid(nb, (C / 8 + 63) / 64);
  colsum_bf16_partial_kernel<<<grid, 256, 0, st>>>((const bf16_t*)m, part, rows, C, rpb);
  orion_colsum_partials2(part, part + (size_t)nb * C, out, nb, C, out_f32, st);
  return (int)hipGetLastError();
}

// part[P][C] partials; mid: COLSUM_SPLITS * C floats of scratch; out fp32 when f32
int orion_colsum_partials2(const float* part, float* mid, void* out, int P, int C, int f32,
                           hipStream_t st) {
  if (!colsum_two_stage()) {
    const ColsumOuts o{{out, nullptr, nullptr}, f32};
    colsum_onepass_kernel<COLSUM_NW, COLSUM_CW><<<dim3((C + COLSUM_CW - 1) / COLSUM_CW, 1), COLSUM_NW * 64, 0, st>>>(part, 0, P, C, o);
    return (int)hipGetLastError();
  }
  const int S = P < COLSUM_SPLITS ? (P < 1 ? 1 : P) : COLSUM_SPLITS;
  const int rps = (P + S - 1) / S;
  colsum_stage1_kernel<<<dim3((C + 63) / 64, S), 256, 0, st>>>(part, mid, P, C, rps);
  colsum_stage2_kernel<<<(C + 255) / 256, 256, 0, st>>>(mid, out, S, C, f32);
  return (int)hipGetLastError();
}

int orion_colsum_scratch(int rows, int C) {  // floats of scratch a colsum of `rows` rows needs
  return (orion_layernorm_bwd_blocks(rows) + 2 * COLSUM_SPLITS) * C;
}
