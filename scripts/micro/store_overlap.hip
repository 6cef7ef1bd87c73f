// Microbenchmark: does one workgroup's epilogue store burst overlap a co-resident workgroup's
// MFMA + LDS-DMA stream on gfx950, and is the burst bound per CU or by the chip's write rate?
//
// Each workgroup (4 waves, 72 KB LDS -> 2 per CU) walks `items` work items; an item is
// `steps` steps of {barrier, 6 LDS-DMA pieces of 1 KB per wave, 32 v_mfma_f32_16x16x32_bf16
// into 32 accumulators} followed (flags & 2) by the fused-GEMM epilogue's stores: 32 x 16 B per
// lane per wave in the gemm16 pattern (16 rows x 64 B per instruction) into a [M][N] bf16
// output.  flags: 1 DMA on, 2 stores on, 4 odd half of the grid starts half an item late
// (extra half item of compute first), 8 stores waited for two steps later (vmcnt(6 + 32)
// for the two steps after an epilogue), 16 only every 8th workgroup runs (the rest exit).
// Build: hipcc -O3 --offload-arch=gfx950 -o /tmp/store_overlap store_overlap.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8m;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

__global__ __launch_bounds__(256, 2) void kern(const unsigned short* __restrict__ src, unsigned short* dst,
                                               int M, int N, int items, int steps, int flags,
                                               unsigned long* cyc) {
  extern __shared__ __attribute__((aligned(16))) unsigned short smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nwg = gridDim.x, bid = blockIdx.x;
  if ((flags & 16) && ((bid >> 3) & 7)) return;
  // register operands: random bf16 from src (not zeros: DVFS)
  bf16x8m a[4], b[8];
  const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
  for (int i = 0; i < 4; ++i) a[i] = __builtin_bit_cast(bf16x8m, s4[(bid * 256 + tid) * 12 + i]);
  for (int i = 0; i < 8; ++i) b[i] = __builtin_bit_cast(bf16x8m, s4[(bid * 256 + tid) * 12 + 4 + i]);
  f32x4 acc[8][4];
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 64 << 20, 0x00020000);
  const int tiles_n = N / 256, tiles = (M / 128) * tiles_n;
  const int late = (flags & 4) && bid >= nwg / 2;
  unsigned long t_store = 0, t0 = __builtin_amdgcn_s_memtime();
  int s = 0;
  int since_epi = 100;
  auto step = [&](bool zero) {
    if (zero) {
      for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if ((flags & 8) && since_epi < 2) wait_vm<6 + 32>();
    else wait_vm<6>();
    __builtin_amdgcn_s_barrier();
    if (flags & 1) {
      unsigned short* base = smem + (s % 3) * 12288;
      const unsigned voff = (unsigned)(((bid * 7919u + s * 24u + w * 6u) & 0xFFF) * 1024u) + lane * 16u;
      for (int e = 0; e < 6; ++e)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(base + w * 3072 + e * 512),
                                                 16, voff + e * 1024, 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[i], a[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    ++s;
    ++since_epi;
  };
  if (late)
    for (int t = 0; t < steps / 2; ++t) step(t == 0);
  for (int it = 0; it < items; ++it) {
    const int tile = bid + it * nwg;
    if (tile >= tiles) break;
    for (int t = 0; t < steps; ++t) step(t == 0);
    if (flags & 2) {
      const unsigned long ts = __builtin_amdgcn_s_memtime();
      const int m0 = (tile / tiles_n) * 128, n0 = (tile % tiles_n) * 256;
      const int wn = w >> 1, wm = w & 1, q = lane >> 4, i16 = lane & 15;
      const int mw = m0 + wm * 64, nw = n0 + wn * 128;
      const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(dst + (long)m0 * N, (short)0, 128 * N * 2, 0x00020000);
      const __amdgpu_buffer_rsrc_t ro2 = __builtin_amdgcn_make_buffer_rsrc(dst + (long)M * N + (long)m0 * N, (short)0, 128 * N * 2, 0x00020000);
      // store pattern: R rows x (64 / R) lanes per row per instruction ((flags >> 8) & 7 = log2 R;
      // 4 = the gemm16 epilogue's 16 rows x 64 B)
      const int lr = (flags >> 8) & 7, R = 1 << lr, L = 64 >> lr;
      const int row_l = lane / L, colb_l = 16 * (lane % L);
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int nblk = 256 / (16 * L);             // instructions across the wave's 256-byte rows
        const int r0 = (k / nblk) * R, c0 = (k % nblk) * 16 * L;
        const int m = mw + r0 + row_l;
        u32x4 pk;
        for (int e = 0; e < 4; ++e) pk[e] = __float_as_uint(acc[k & 7][(k >> 3) * 2][e]) ^ __float_as_uint(acc[k & 7][(k >> 3) * 2 + 1][e]);
        const unsigned off = (unsigned)((m - m0) * N * 2 + nw * 2 + c0 + colb_l);
        // cache-policy bits of the stores ((flags >> 12) & 7): 0 none, 1 nt (aux 2), 2 sc1 (16),
        // 3 nt | sc1 (18), 4 sc0 (1), 5 sc0 | nt (3)
        switch ((flags >> 12) & 7) {
#define ST(AUX) __builtin_amdgcn_raw_buffer_store_b128(pk, ro, off, 0, AUX); __builtin_amdgcn_raw_buffer_store_b128(pk, ro2, off, 0, AUX); break;
          case 1: ST(2)
          case 2: ST(16)
          case 3: ST(18)
          case 4: ST(1)
          case 5: ST(3)
          default: ST(0)
#undef ST
        }
      }
      t_store += __builtin_amdgcn_s_memtime() - ts;
      since_epi = 0;
    }
  }
  wait_vm<0>();
  const unsigned long t1 = __builtin_amdgcn_s_memtime();
  if (!(flags & 2)) {  // keep the accumulators alive
    float z = 0.f;
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 4; ++j) z += acc[i][j][0];
    if (z == 12345.678f) dst[tid] = 1;
  }
  if (lane == 0) {
    cyc[(bid * 4 + w) * 2] = t1 - t0;
    cyc[(bid * 4 + w) * 2 + 1] = t_store;
  }
}

int main(int argc, char** argv) {
  const int M = 65536, N = 3072, steps = argc > 1 ? atoi(argv[1]) : 24;
  const size_t srcb = 64 << 20, dstb = (size_t)2 * M * N * 2;
  unsigned short *src, *dst;
  unsigned long* cyc;
  CK(hipMalloc(&src, srcb));
  CK(hipMalloc(&dst, dstb));
  CK(hipMalloc(&cyc, 1024 * 4 * 2 * 8));
  std::vector<unsigned short> h(srcb / 2);
  unsigned x = 12345;
  for (auto& v : h) { x = x * 1664525u + 1013904223u; v = (unsigned short)(0x3C00 | ((x >> 9) & 0x83FF)); }
  CK(hipMemcpy(src, h.data(), srcb, hipMemcpyHostToDevice));
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Cfg { const char* name; int grid, flags; };
  const int tiles = (M / 128) * (N / 256);
  std::vector<Cfg> cfgs;
  const char* pn[7] = {"1 row x 1 KB", "", "4 rows x 256 B", "8 rows x 128 B", "16 rows x 64 B (gemm16)", "", "64 rows x 16 B"};
  const char* an[6] = {"plain", "nt", "sc1", "nt|sc1", "sc0", "sc0|nt"};
  static char names[64][96];
  int ni = 0;
  snprintf(names[ni], 96, "MFMA+DMA (no stores)");
  cfgs.push_back({names[ni++], 512, 1});
  for (int lr : {4, 3, 0}) {
    for (int a : {0, 1, 2, 3, 4, 5}) {
      snprintf(names[ni], 96, "MFMA+DMA+stores deferred %s %s", pn[lr], an[a]);
      cfgs.push_back({names[ni++], 512, 11 | (lr << 8) | (a << 12)});
    }
  }
  snprintf(names[ni], 96, "MFMA+DMA (no stores)");
  cfgs.push_back({names[ni++], 512, 1});
  std::vector<unsigned long> hc(1024 * 8);
  for (int rep = 0; rep < 1; ++rep) {
    for (auto& c : cfgs) {
      const int items = (tiles + c.grid - 1) / c.grid;
      const int lds = c.grid == 256 ? 96 * 1024 : 72 * 1024;  // 96 KB: one workgroup per CU
      std::vector<float> ms;
      for (int i = 0; i < 7; ++i) {
        CK(hipEventRecord(e0));
        kern<<<c.grid, 256, lds>>>(src, dst, M, N, items, steps, c.flags, cyc);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
      }
      std::sort(ms.begin(), ms.end());
      CK(hipMemcpy(hc.data(), cyc, c.grid * 4 * 2 * 8, hipMemcpyDeviceToHost));
      std::vector<double> tot, st;
      for (int b = 0; b < c.grid; ++b) {
        if ((c.flags & 16) && ((b >> 3) & 7)) continue;
        tot.push_back((double)hc[b * 8]);
        st.push_back((double)hc[b * 8 + 1]);
      }
      std::sort(tot.begin(), tot.end());
      std::sort(st.begin(), st.end());
      const double flop = 2.0 * M * N * 32.0 * steps * ((c.flags & 16) ? 0.125 : 1.0);
      printf("{\"cfg\": \"%s\", \"steps\": %d, \"ms\": %.4f, \"TFs_equiv\": %.1f, \"wave_cycles_med\": %.0f, \"store_issue_cycles_med\": %.0f, \"clk_GHz_est\": %.3f}\n",
             c.name, steps, ms[3], flop / ms[3] / 1e9, tot[tot.size() / 2], st[st.size() / 2],
             tot[tot.size() / 2] / (ms[3] * 1e6));
    }
  }
  return 0;
}
