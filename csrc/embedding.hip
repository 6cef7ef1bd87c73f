// Embedding backward straight into the fp32 gradient arena (gfx950).
//
// GPT-2's token table is tied to the LM head: the LM head's weight gradient is written into
// the table's fp32 arena slice first (the first op of the backward), the embedding's
// contribution last.  Instead of autograd's dense path for it (a zero-filled [V, C]
// gradient, a sort of the token ids, a segmented sum, then a bf16 add into the LM head's
// gradient and an fp32 fold into the arena: ~0.45 ms per GPT-2 step, on the critical path of
// the last data-parallel bucket), every token row of dx is added into its table row with
// fp32 atomics, one 16-byte chunk of dx per lane (global_atomic_add_f32, -munsafe-fp-atomics).
// The summation order over duplicate tokens is not fixed, so deterministic mode
// (ops/determinism.py) keeps the sort-based path.
#include "common.h"

namespace orion {

// out[idx[row]][c] += dx[row][c]: one wave per row, lane l adding columns l, l + 64, ... so
// every atomic instruction covers 64 consecutive floats (two 128-byte lines) -- the
// chunk-per-lane layout (eight scattered 32-byte-strided atomics per instruction) ran 4x
// slower
__global__ __launch_bounds__(256) void embed_scatter_add_kernel(const bf16_t* __restrict__ dx,
                                                                const int64_t* __restrict__ idx,
                                                                float* __restrict__ out, long rows,
                                                                int C, long V, int* err) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const long id = idx[row];
  ORION_DASSERT(id >= 0 && id < V);
  if ((unsigned long)id >= (unsigned long)V) {  // never an atomic outside the table: flag it
    if (lane == 0) atomicOr(err, 1);
    return;
  }
  const bf16_t* d = dx + row * C;
  float* o = out + id * C;
  for (int c = lane; c < C; c += 64) atomicAdd(o + c, bf2f(d[c]));
}

// out[j] = sum_b x[b][j] over B rows of n elements (the position table's gradient: dx summed
// over the batch), 8 columns per thread, fixed summation order; out fp32 or bf16
__global__ __launch_bounds__(256) void batch_sum_kernel(const bf16_t* __restrict__ x, void* __restrict__ out,
                                                        int B, long n, int f32) {
  const long j = ((long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (j >= n) return;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int b = 0; b < B; ++b) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (long)b * n + j);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += bf2f(v[k]);
  }
  if (f32) {
    f32x4* o = reinterpret_cast<f32x4*>(static_cast<float*>(out) + j);
    o[0] = f32x4{acc[0], acc[1], acc[2], acc[3]};
    o[1] = f32x4{acc[4], acc[5], acc[6], acc[7]};
  } else {
    bf16x8 r;
#pragma unroll
    for (int k = 0; k < 8; ++k) r[k] = f2bf(acc[k]);
    *reinterpret_cast<bf16x8*>(static_cast<bf16_t*>(out) + j) = r;
  }
}

}  // namespace orion

using namespace orion;

extern "C++" {

int orion_embed_scatter_add(const void* dx, const int64_t* idx, float* out, long rows, int C,
                            long V, int* err, hipStream_t st) {
  if (rows == 0) return 0;
  embed_scatter_add_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>((const bf16_t*)dx, idx, out,
                                                                        rows, C, V, err);
  return (int)hipGetLastError();
}

int orion_batch_sum(const void* x, void* out, int B, long n, int out_f32, hipStream_t st) {
  if (n % 8 != 0) return -1;
  if (n == 0) return 0;
  batch_sum_kernel<<<(unsigned)((n / 8 + 255) / 256), 256, 0, st>>>((const bf16_t*)x, out, B, n, out_f32);
  return (int)hipGetLastError();
}

}  // extern "C++"
