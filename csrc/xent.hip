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

namespace orion {

constexpr int XT = 512;  // threads per row
constexpr int XW = XT / 64;

// inv_n[0] = 1 / max(1, #targets != ignore_index)
__global__ __launch_bounds__(256) void count_valid_kernel(const int64_t* __restrict__ t, long N,
                                                          long ignore, float* __restrict__ inv_n) {
  __shared__ float red[4];
  float c = 0.f;
  for (long i = threadIdx.x; i < N; i += 256) c += (t[i] != ignore) ? 1.f : 0.f;
  c = block_sum<4>(c, red);
  if (threadIdx.x == 0) inv_n[0] = 1.f / fmaxf(c, 1.f);
}

template <int CH>  // 16-byte chunks per thread (CH * 8 * XT >= V)
__global__ __launch_bounds__(XT) void xent_fwd_bwd_kernel(
    bf16_t* __restrict__ logits, const int64_t* __restrict__ targets, float* __restrict__ losses,
    const float* __restrict__ inv_n, int V, long ignore) {
  __shared__ float red[XW];
  const long row = blockIdx.x;
  bf16_t* lr = logits + row * (long)V;
  const int V8 = V >> 3;
  bf16x8 v[CH];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = k * XT + threadIdx.x;
    if (c < V8) {
      v[k] = *reinterpret_cast<const bf16x8*>(lr + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, bf2f(v[k][j]));
    }
  }
  m = block_max<XW>(m, red);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = k * XT + threadIdx.x;
    if (c < V8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(bf2f(v[k][j]) - m);
    }
  }
  s = block_sum<XW>(s, red);
  const long tgt = targets[row];
  const bool valid = tgt != ignore;
  const float lse = m + __logf(s);
  const float scale = valid ? inv_n[0] : 0.f;
  const float inv_s = 1.f / s;
  if (threadIdx.x == 0) {
    losses[row] = valid ? (lse - bf2f(lr[tgt])) : 0.f;
  }
  __syncthreads();  // the target logit is read above before anyone overwrites it
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = k * XT + threadIdx.x;
    if (c < V8) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float p = __expf(bf2f(v[k][j]) - m) * inv_s;
        if (c * 8 + j == tgt) p -= 1.f;
        o[j] = f2bf(p * scale);
      }
      *reinterpret_cast<bf16x8*>(lr + c * 8) = o;
    }
  }
}

// loss = sum(losses) * inv_n   (single workgroup, deterministic order)
__global__ __launch_bounds__(1024) void mean_loss_kernel(const float* __restrict__ losses, long N,
                                                         const float* __restrict__ inv_n,
                                                         float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (long i = threadIdx.x; i < N; i += 1024) s += losses[i];
  s = block_sum<16>(s, red);
  if (threadIdx.x == 0) out[0] = s * inv_n[0];
}

}  // namespace orion

using namespace orion;

// logits (N, V) bf16 is overwritten with dlogits; scratch: losses[N] fp32, inv_n[1] fp32.
int orion_xent_fwd_bwd(void* logits, const int64_t* targets, float* losses, float* inv_n,
                       float* loss_out, long N, int V, long ignore, hipStream_t st) {
  if (V % 8) return -1;
  count_valid_kernel<<<1, 256, 0, st>>>(targets, N, ignore, inv_n);
  const int chunks = (V / 8 + XT - 1) / XT;
  auto L = (bf16_t*)logits;
  switch (chunks) {
#define XC(K) case K: xent_fwd_bwd_kernel<K><<<N, XT, 0, st>>>(L, targets, losses, inv_n, V, ignore); break;
    XC(1) XC(2) XC(3) XC(4) XC(5) XC(6) XC(7) XC(8) XC(9) XC(10) XC(11) XC(12) XC(13) XC(14)
    XC(15) XC(16) XC(17) XC(18) XC(19) XC(20) XC(21) XC(22) XC(23) XC(24) XC(25) XC(26)
    XC(27) XC(28) XC(29) XC(30) XC(31) XC(32)
#undef XC
    default: return -2;  // V > 131072
  }
  mean_loss_kernel<<<1, 1024, 0, st>>>(losses, N, inv_n, loss_out);
  return (int)hipGetLastError();
}
