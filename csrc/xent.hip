// Fused softmax cross-entropy forward+backward (K9 in SURVEY.md §2.11).
//
// One workgroup (512 threads = 8 waves) per row of the (N, V) bf16 logits.
// The row (V = 50304 for GPT-2: ~100 KB) is read from HBM ONCE into registers
// (13 x 16-byte vectors per lane), the max/sum-exp are reduced across the 8
// waves, and the gradient  dlogits = (softmax - onehot(target)) / n_valid  is
// written IN PLACE over the logits.  Training always runs backward after the
// loss, so computing the gradient here saves a second full read of the logits
// and the fp32 probability tensor a separate softmax would materialise.
// The caller (``ops/xent.py``) multiplies by the upstream gradient afterwards
// on the much smaller GEMM outputs.
#include "common.h"
#include "mfma_lds.h"

// cache-policy bits of the row's buffer loads / stores (A/B builds: -DXENT_LD_AUX=..)
#ifndef XENT_LD_AUX
#define XENT_LD_AUX 2  // nt: the row is streamed once (2.34 vs 2.66 ms per GPT-2 step, profiles/ab/xent_nt_r04.log)
#endif
#ifndef XENT_ST_AUX
#define XENT_ST_AUX 2
#endif

namespace orion {


// inv_n[0] = 1 / max(1, #valid targets).  A target is valid when it is not ignore_index and
// lies in [0, V) (the same rule as csrc/lmhead.hip's lm_valid); any other target is skipped
// (no loss, no gradient) and raises the device flag ``err`` (ops.embedding.id_error, where
// torch's cross_entropy would raise).  One workgroup; 8 independent loads in flight per
// thread so the pass is bandwidth- not latency-bound.
__device__ __forceinline__ void tgt_count(long v, long ignore, int V, float& c, float& bad) {
  const bool in = v >= 0 && v < V;
  c += (v != ignore && in) ? 1.f : 0.f;
  bad += (v != ignore && !in) ? 1.f : 0.f;
}

template <typename T>  // i64x2 when the targets are 16-byte aligned, else int64_t
__global__ __launch_bounds__(1024) void count_valid_kernel(const int64_t* __restrict__ t, long N,
                                                           long ignore, int V, float* __restrict__ inv_n,
                                                           int* __restrict__ err) {
  __shared__ float red[16];
  constexpr int PER = sizeof(T) / sizeof(int64_t);
  const long NV = N / PER;
  const T* tv = reinterpret_cast<const T*>(t);
  float c = 0.f, bad = 0.f;
  for (long base = threadIdx.x; base < NV; base += 8 * 1024) {
    T v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long i = base + u * 1024;
      if (i < NV) v[u] = tv[i];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (base + u * 1024 < NV) {
        if constexpr (PER == 2) {
          tgt_count(v[u][0], ignore, V, c, bad);
          tgt_count(v[u][1], ignore, V, c, bad);
        } else {
          tgt_count(v[u], ignore, V, c, bad);
        }
      }
  }
  if (threadIdx.x == 0)
    for (long i = NV * PER; i < N; ++i) tgt_count(t[i], ignore, V, c, bad);
  c = block_sum<16>(c, red);
  bad = block_sum<16>(bad, red);
  if (threadIdx.x == 0) {
    inv_n[0] = 1.f / fmaxf(c, 1.f);
    if (bad > 0.f) err[0] = 1;
  }
}

// Occupancy: the row lives in registers (CH x 4 VGPRs), so the VGPR budget decides how
// many rows a CU streams at once: while one row is in its reduction phase the others are
// loading/storing, which is what keeps HBM busy (one row per CU left it ~50% idle).  The
// row is addressed through one buffer resource (chunk step in the scalar offset), which
// takes the kernel from 86 to 72 VGPRs: THREE 8-wave workgroups per CU instead of two.
// Vocabularies over 13 x 4096 use 1024 threads per row so CH stays <= 13.
template <int CH, int XT>  // 16-byte chunks per thread (CH * 8 * XT >= V)
__global__ __launch_bounds__(XT, (XT == 512 ? 4 : 2)) void xent_fwd_bwd_kernel(
    bf16_t* __restrict__ logits, const int64_t* __restrict__ targets, float* __restrict__ losses,
    const float* __restrict__ inv_n, int V, long ignore) {
  constexpr int XW = XT / 64;
  constexpr float L2E = 1.4426950408889634f;
  __shared__ float red[XW];
  const long row = blockIdx.x;
  bf16_t* lr = logits + row * (long)V;
  const int V8 = V >> 3;
  // the row through one buffer resource: a lane's 16-byte chunk offset in a VGPR, the chunk
  // step k * XT * 16 in the scalar offset (no per-lane 64-bit address per chunk)
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(lr, (unsigned)V * 2);
  const unsigned vo = threadIdx.x * 16;
  bf16x8 v[CH];
  // pass 1: row max (max3 chains; this file builds with -fno-honor-nans, so fmaxf needs no
  // canonicalising max per operand)
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = k * XT + threadIdx.x;
    if (c < V8) {
      v[k] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rr, vo, k * XT * 16, XENT_LD_AUX));
      float a = fmaxf(fmaxf(bf2f(v[k][0]), bf2f(v[k][1])), bf2f(v[k][2]));
      a = fmaxf(fmaxf(a, bf2f(v[k][3])), bf2f(v[k][4]));
      a = fmaxf(fmaxf(a, bf2f(v[k][5])), bf2f(v[k][6]));
      m = fmaxf(fmaxf(m, a), bf2f(v[k][7]));
    }
  }
  m = block_max<XW>(m, red);
  // pass 2: e = exp(x - m) as one fma + v_exp (base 2), kept in the registers as bf16 (the
  // output is bf16 anyway) so pass 3 does not recompute it; four sum chains
  const float m2 = m * L2E;
  const long tgt = targets[row];
  const bool valid = tgt != ignore && tgt >= 0 && tgt < V;  // see count_valid_kernel
  // the thread whose 16-byte chunks hold the target logit owns the loss (one scalar
  // re-read of that logit; a per-element compare against the target would cost a select
  // per logit)
  const bool owner = valid && (int)((tgt >> 3) % XT) == (int)threadIdx.x;
  const float xt = owner ? bf2f(lr[tgt]) : 0.f;
  float s4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = k * XT + threadIdx.x;
    if (c < V8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float e = __builtin_amdgcn_exp2f(fmaf(bf2f(v[k][j]), L2E, -m2));
        s4[j & 3] += e;
        v[k][j] = f2bf(e);
      }
    }
  }
  const float s = block_sum<XW>((s4[0] + s4[1]) + (s4[2] + s4[3]), red);
  const float lse = m + __logf(s);
  const float scale = valid ? inv_n[0] : 0.f;
  const float f = scale / s;
  if (!valid && threadIdx.x == 0) losses[row] = 0.f;
  // pass 3: dlogits = (softmax - onehot) / n_valid in place
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = k * XT + threadIdx.x;
    if (c < V8) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(v[k][j]) * f);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rr, vo, k * XT * 16, XENT_ST_AUX);
    }
  }
  if (owner) {  // the target's own term (after this thread's store of its chunk)
    lr[tgt] = f2bf(__builtin_amdgcn_exp2f(fmaf(xt, L2E, -m2)) * f - scale);
    losses[row] = lse - xt;
  }
}

// loss = sum(losses) * inv_n   (single workgroup, deterministic order)
__global__ __launch_bounds__(1024) void mean_loss_kernel(const float* __restrict__ losses, long N,
                                                         const float* __restrict__ inv_n,
                                                         float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (long base = threadIdx.x; base < N; base += 8 * 1024) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = base + u * 1024 < N ? losses[base + u * 1024] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  s = block_sum<16>(s, red);
  if (threadIdx.x == 0) out[0] = s * inv_n[0];
}

}  // namespace orion

using namespace orion;

// logits (N, V) bf16 is overwritten with dlogits; scratch: losses[N] fp32, inv_n[1] fp32.
int orion_xent_fwd_bwd(void* logits, const int64_t* targets, float* losses, float* inv_n,
                       float* loss_out, long N, int V, long ignore, int* err, hipStream_t st) {
  if (V % 8) return -1;
  if ((reinterpret_cast<uintptr_t>(targets) & 15) == 0)
    count_valid_kernel<i64x2><<<1, 1024, 0, st>>>(targets, N, ignore, V, inv_n, err);
  else
    count_valid_kernel<int64_t><<<1, 1024, 0, st>>>(targets, N, ignore, V, inv_n, err);
  auto L = (bf16_t*)logits;
  const int c512 = (V / 8 + 511) / 512, c1024 = (V / 8 + 1023) / 1024;
  if (c512 <= 13) {
    switch (c512) {
#define XC(K) case K: xent_fwd_bwd_kernel<K, 512><<<N, 512, 0, st>>>(L, targets, losses, inv_n, V, ignore); break;
      XC(1) XC(2) XC(3) XC(4) XC(5) XC(6) XC(7) XC(8) XC(9) XC(10) XC(11) XC(12) XC(13)
#undef XC
    }
  } else {
    switch (c1024) {
#define XC(K) case K: xent_fwd_bwd_kernel<K, 1024><<<N, 1024, 0, st>>>(L, targets, losses, inv_n, V, ignore); break;
      XC(7) XC(8) XC(9) XC(10) XC(11) XC(12) XC(13) XC(14) XC(15) XC(16)
#undef XC
      default: return -2;  // V > 131072
    }
  }
  mean_loss_kernel<<<1, 1024, 0, st>>>(losses, N, inv_n, loss_out);
  return (int)hipGetLastError();
}
