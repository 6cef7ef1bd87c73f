// LM head + softmax cross-entropy without a pass over the logits (K9 in SURVEY.md §2.11;
// VERDICT r4 item 2).  Round 4 computed the (N, V) logits with a GEMM, then ran a row pass
// (csrc/xent.hip) that read them and wrote dlogits back in place: 13 GB of HBM traffic
// (2.3 ms per GPT-2 step) between the forward GEMM and the two backward GEMMs.  Here:
//
//   forward GEMM (gemm16 EPI_EXP)  E[m][n] = exp(l[m][n] - C)  (bf16, the buffer the logits
//       used), per-(row, 128-column) fp32 partial sums of E, and l[m][t_m] (fp32) -- C is one
//       device scalar, the largest row log-sum-exp of the previous call;
//   fold (this file)  Z_m = sum of the partials, lse_m = C + ln Z_m, loss_m = lse_m - l[m][t_m],
//       and the one-hot term folded into the exp tile: E[m][t_m] <- exp(l[m][t_m] - C) - Z_m,
//       so that s_m E'[m] = dlogits[m] with s_m = g / (Z_m n_valid);
//   rows whose Z_m is not a normal number of moderate size (a logit more than ~60 above C
//       overflows, a row whose every logit sits ~80 below C underflows) are recomputed from
//       x and W with their own reference (fixup: a GEMV per such row, rare by construction);
//   backward  dX = s (E' W)  (gemm16 EPI_ROWSCALE: the row scale in the epilogue) and
//       dW = E'^T (s X)  (the plain weight-gradient GEMM on X pre-scaled per row).
//
// The only passes left besides the three GEMMs read the (N, V / 128) partials (103 MB at
// GPT-2's shape) and the (N, C) activations.
#include "common.h"

namespace orion {

constexpr float LM_L2E = 1.4426950408889634f;
// Z_m outside [2^-100, 2^100]: recompute the row (its largest term lost precision or
// overflowed against the shared reference)
constexpr float LM_ZMIN = 7.888609052210118e-31f, LM_ZMAX = 1.2676506002282294e30f;

ORION_DEVICE bool lm_valid(long t, long ignore, int V) { return t != ignore && t >= 0 && t < V; }

// One wave per row: Z, lse, loss, the one-hot fold; rows to recompute go to fix_list.  (The
// valid-row count is the finalize kernel's: one global atomic per workgroup here -- 16,384 of
// them on one address at GPT-2's shape -- serialised the kernel to ~0.19 ms.)
__global__ __launch_bounds__(256) void lmhead_fold_kernel(
    const float* __restrict__ part, int npart, const float* __restrict__ tlog,
    const int64_t* __restrict__ tgt, long ignore, const float* __restrict__ cref, bf16_t* E,
    long lde, int V, int N, float* __restrict__ invz, float* __restrict__ lse,
    float* __restrict__ loss, int* __restrict__ counts, int* __restrict__ fix_list) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row < N) {
    const float* pr = part + row * npart;
    float z = 0.f;
    if (npart <= 512) {
      // every load of the row in flight at once (a loop paid the load latency per iteration:
      // the fold ran at ~0.5 TB/s); fixed summation order
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = lane + 64 * k < npart ? pr[lane + 64 * k] : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) z += v[k];
    } else {
      for (int i = lane; i < npart; i += 64) z += pr[i];
    }
    z = wave_sum(z);
    const long t = tgt[row];
    const bool valid = lm_valid(t, ignore, V);
    const float c = *cref;
    const bool fix = !(z >= LM_ZMIN && z <= LM_ZMAX);  // NaN / inf / 0 too
    if (lane == 0) {
      if (fix) {
        fix_list[atomicAdd(&counts[1], 1)] = (int)row;
      } else {
        invz[row] = 1.f / z;
        lse[row] = c + __logf(z);
        if (valid) {
          const float lt = tlog[row];
          loss[row] = c + __logf(z) - lt;
          E[row * lde + t] = f2bf(__builtin_amdgcn_exp2f((lt - c) * LM_L2E) - z);
        } else {
          loss[row] = 0.f;
        }
      }
    }
  }
}

// Rows flagged by the fold: logits recomputed as a GEMV against W (two passes: the row max,
// then exp / sum / store), the row's own reference.  A fixed grid walks the list (counts[1]
// entries); with none it exits at once.
__global__ __launch_bounds__(256) void lmhead_fixup_kernel(
    const bf16_t* __restrict__ X, long ldx, const bf16_t* __restrict__ W, long ldw, int Cdim, int V,
    const float* __restrict__ tlog, const int64_t* __restrict__ tgt, long ignore, bf16_t* E, long lde,
    float* __restrict__ invz, float* __restrict__ lse, float* __restrict__ loss,
    const int* __restrict__ counts, const int* __restrict__ fix_list) {
  extern __shared__ __attribute__((aligned(16))) float xs[];  // Cdim floats
  __shared__ float red[4];
  const int nfix = counts[1];
  for (int i = blockIdx.x; i < nfix; i += gridDim.x) {
    const long row = fix_list[i];
    __syncthreads();
    for (int k = threadIdx.x; k < Cdim; k += 256) xs[k] = bf2f(X[row * ldx + k]);
    __syncthreads();
    auto logit = [&](int n) {
      const bf16_t* wr = W + (long)n * ldw;
      float a = 0.f;
      for (int k = 0; k < Cdim; k += 8) {
        const bf16x8 w8 = *reinterpret_cast<const bf16x8*>(wr + k);
#pragma unroll
        for (int j = 0; j < 8; ++j) a = fmaf(xs[k + j], bf2f(w8[j]), a);
      }
      return a;
    };
    float mx = -INFINITY;
    for (int n = threadIdx.x; n < V; n += 256) mx = fmaxf(mx, logit(n));
    mx = block_max<4>(mx, red);
    float z = 0.f;
    for (int n = threadIdx.x; n < V; n += 256) {
      const float e = __builtin_amdgcn_exp2f((logit(n) - mx) * LM_L2E);
      z += e;
      E[row * lde + n] = f2bf(e);
    }
    z = block_sum<4>(z, red);  // its barriers order the row's stores before the fold below
    if (threadIdx.x == 0) {
      const long t = tgt[row];
      invz[row] = 1.f / z;
      lse[row] = mx + __logf(z);
      if (lm_valid(t, ignore, V)) {
        const float lt = tlog[row];
        loss[row] = mx + __logf(z) - lt;
        E[row * lde + t] = f2bf(__builtin_amdgcn_exp2f((lt - mx) * LM_L2E) - z);
      } else {
        loss[row] = 0.f;
      }
    }
  }
}

// loss = sum(loss_m) / n_valid (fixed order), inv_n, and the next call's reference: the
// largest finite row lse (keeps every row's exp at most ~1 for the next weights).
__global__ __launch_bounds__(1024) void lmhead_finalize_kernel(const float* __restrict__ loss_rows,
                                                               const float* __restrict__ lse, long N,
                                                               const int64_t* __restrict__ tgt, long ignore,
                                                               int V, float* __restrict__ out,
                                                               float* __restrict__ inv_n, float* __restrict__ cref,
                                                               int* __restrict__ err) {
  __shared__ float red[16];
  float s = 0.f, mx = -INFINITY, nv = 0.f, bad = 0.f;
  for (long i = threadIdx.x; i < N; i += 1024) {
    s += loss_rows[i];
    const float l = lse[i];
    if (l == l && l < INFINITY) mx = fmaxf(mx, l);
    const long t = tgt[i];
    nv += lm_valid(t, ignore, V) ? 1.f : 0.f;
    bad += (t != ignore && !lm_valid(t, ignore, V)) ? 1.f : 0.f;
  }
  s = block_sum<16>(s, red);
  mx = block_max<16>(mx, red);
  nv = block_sum<16>(nv, red);  // exact: integer counts below 2^24 per lane sum
  bad = block_sum<16>(bad, red);
  if (threadIdx.x == 0) {
    if (bad > 0.f) err[0] = 1;  // an out-of-range target (not ignore_index): skipped, flagged
    const float in = 1.f / fmaxf(nv, 1.f);
    inv_n[0] = in;
    out[0] = s * in;
    if (mx > -INFINITY) cref[0] = mx;
  }
}

// Backward prologue: s_m = g / (Z_m n_valid) for valid rows (0 otherwise) and Xs = s (.) X.
__global__ __launch_bounds__(256) void lmhead_bwd_prep_kernel(
    const bf16_t* __restrict__ X, long ldx, int Cdim, long N, const int64_t* __restrict__ tgt, long ignore,
    int V, const float* __restrict__ invz, const float* __restrict__ inv_n, const float* __restrict__ g,
    float* __restrict__ srow, bf16_t* __restrict__ Xs) {
  const int c8 = Cdim / 8;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= N * c8) return;
  const long row = i / c8;
  const int k = (int)(i - row * c8) * 8;
  const float s = lm_valid(tgt[row], ignore, V) ? g[0] * inv_n[0] * invz[row] : 0.f;
  if (k == 0) srow[row] = s;
  const bf16x8 x = *reinterpret_cast<const bf16x8*>(X + row * ldx + k);
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(x[j]) * s);
  *reinterpret_cast<bf16x8*>(Xs + row * Cdim + k) = o;
}

// The same with Xs written transposed, XsT [Cdim][N] (N % 64 == 0, Cdim % 64 == 0): the
// weight gradient dW = E'^T Xs then reads Xs as an NT operand (one ds_read_b128 per fragment
// instead of two transposing reads, csrc/wgrad.hip orion_wgrad_nt).  One 64-row x 64-column
// block per workgroup, transposed through LDS.
__global__ __launch_bounds__(256) void lmhead_bwd_prep_t_kernel(
    const bf16_t* __restrict__ X, long ldx, long N, const int64_t* __restrict__ tgt, long ignore, int V,
    const float* __restrict__ invz, const float* __restrict__ inv_n, const float* __restrict__ g,
    float* __restrict__ srow, bf16_t* __restrict__ XsT) {
  __shared__ bf16_t tile[64][64 + 8];  // [column][row]
  const int tid = threadIdx.x;
  const long r0 = (long)blockIdx.x * 64;
  const int c0 = blockIdx.y * 64;
  {
    const int r = tid >> 2, cc = (tid & 3) * 16;
    const long row = r0 + r;
    const float sv = lm_valid(tgt[row], ignore, V) ? g[0] * inv_n[0] * invz[row] : 0.f;
    if (blockIdx.y == 0 && (tid & 3) == 0) srow[row] = sv;
    const bf16x8* src = reinterpret_cast<const bf16x8*>(X + row * ldx + c0 + cc);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const bf16x8 x = src[h];
#pragma unroll
      for (int j = 0; j < 8; ++j) tile[cc + 8 * h + j][r] = f2bf(bf2f(x[j]) * sv);
    }
  }
  __syncthreads();
  {
    const int c = tid >> 2, rr = (tid & 3) * 16;
    bf16x8* dst = reinterpret_cast<bf16x8*>(XsT + (long)(c0 + c) * N + r0 + rr);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = tile[c][rr + 8 * h + j];
      dst[h] = o;
    }
  }
}

}  // namespace orion

using namespace orion;

// Fold + fixup + finalize after the EPI_EXP GEMM.  counts: int[2] scratch (zeroed here);
// fix_list: int[N]; xs_lds: the fixup's LDS bytes (Cdim floats).
int orion_lmhead_fold(const float* part, int npart, const float* tlog, const int64_t* tgt, long ignore,
                      float* cref, void* E, long lde, int V, long N, const void* X, long ldx, const void* W,
                      long ldw, int Cdim, float* invz, float* lse, float* loss_rows, int* counts,
                      int* fix_list, float* loss_out, float* inv_n, int* err, hipStream_t st) {
  if (N <= 0 || N > 0x7FFFFFFFL || Cdim % 8 || Cdim > 16384) return -1;  // fixup LDS: Cdim floats
  if (hipMemsetAsync(counts, 0, 16, st) != hipSuccess) return -2;
  lmhead_fold_kernel<<<(unsigned)((N + 3) / 4), 256, 0, st>>>(part, npart, tlog, tgt, ignore, cref,
                                                              (bf16_t*)E, lde, V, (int)N, invz, lse,
                                                              loss_rows, counts, fix_list);
  lmhead_fixup_kernel<<<64, 256, Cdim * sizeof(float), st>>>((const bf16_t*)X, ldx, (const bf16_t*)W, ldw,
                                                             Cdim, V, tlog, tgt, ignore, (bf16_t*)E, lde,
                                                             invz, lse, loss_rows, counts, fix_list);
  lmhead_finalize_kernel<<<1, 1024, 0, st>>>(loss_rows, lse, N, tgt, ignore, V, loss_out, inv_n, cref, err);
  return (int)hipGetLastError();
}

// transposed != 0: Xs is written as XsT [Cdim][N] (needs N % 64 == 0 and Cdim % 64 == 0)
int orion_lmhead_bwd_prep(const void* X, long ldx, int Cdim, long N, const int64_t* tgt, long ignore,
                          int V, const float* invz, const float* inv_n, const float* g, float* srow,
                          void* Xs, int transposed, hipStream_t st) {
  if (transposed) {
    if (N % 64 || Cdim % 64 || ldx % 8 || N / 64 > 0x7FFFFFFFL) return -1;
    lmhead_bwd_prep_t_kernel<<<dim3((unsigned)(N / 64), (unsigned)(Cdim / 64)), 256, 0, st>>>(
        (const bf16_t*)X, ldx, N, tgt, ignore, V, invz, inv_n, g, srow, (bf16_t*)Xs);
    return (int)hipGetLastError();
  }
  if (Cdim % 8) return -1;
  const long n = N * (Cdim / 8);
  lmhead_bwd_prep_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(
      (const bf16_t*)X, ldx, Cdim, N, tgt, ignore, V, invz, inv_n, g, srow, (bf16_t*)Xs);
  return (int)hipGetLastError();
}
