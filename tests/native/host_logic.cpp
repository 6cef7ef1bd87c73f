// Host-side logic of the kernel launchers (csrc/*.hip), run under AddressSanitizer and
// UndefinedBehaviorSanitizer on the CPU: split-count planning, scratch sizing and the
// argument validation that must reject a bad call BEFORE anything is launched.  Built by
// tests/test_native_host_sanitizers.py with the sanitizers on the host side only
// (hipcc -Xarch_host -fsanitize=...); no kernel is launched, so no GPU is needed.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

int orion_wgrad_splits(int M, int N1, int N2);
int orion_wgrad_effective_splits(int M, int S);
int orion_wgrad_tail_rows(int M, int N1, int N2, int* S2);
int orion_wgrad(const void*, long, const void*, long, int, int, int, int, float*, void*,
                const float*, int, int, int, hipStream_t);
int orion_gemm(const void*, long, const void*, long, int, int, int, int, int, void*, long,
               const void*, void*, long, const void*, long, hipStream_t, void* db = nullptr,
               int db_f32 = 0, float* part = nullptr);
int orion_gemm_colsum_scratch(int M, int N);
int orion_layernorm_bwd_blocks(int rows);
int orion_colsum_scratch(int rows, int C);
int orion_rmsnorm_bwd_blocks(int rows);

static int failures = 0;
#define CHECK(cond)                                                       \
  do {                                                                    \
    if (!(cond)) {                                                        \
      std::fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #cond); \
      ++failures;                                                         \
    }                                                                     \
  } while (0)

int main() {
  // split-K planning over the shapes the models produce (and odd ones)
  const int Ms[] = {32, 96, 256, 4096, 8192, 8224, 16384, 65536, 131072, 262144};
  const int Ns[] = {8, 64, 264, 768, 1000, 2304, 3072, 4096, 11008, 50304};
  for (int M : Ms)
    for (int n1 : Ns)
      for (int n2 : Ns) {
        const int S = orion_wgrad_splits(M, n1, n2);
        CHECK(S >= 1 && S <= 32);
        CHECK(orion_wgrad_effective_splits(M, S) == S);
        for (int req = 1; req <= 40; req += 3) {
          const int e = orion_wgrad_effective_splits(M, req);
          CHECK(e >= 1 && e <= req);
        }
      }
  // tail split: head rows are the whole tile rows inside the whole rounds, the tail (a partial
  // last tile row allowed) at most half a round
  for (int M : Ms)
    for (int n1 : Ns)
      for (int n2 : Ns) {
        int S2 = 0;
        const int R1 = orion_wgrad_tail_rows(M, n1, n2, &S2);
        CHECK(R1 >= 0 && R1 < n1 && R1 % 256 == 0);
        if (R1 > 0) {
          const long t1 = (n1 + 255) / 256, t2 = (n2 + 255) / 256, tiles = t1 * t2;
          const long head = (long)(R1 / 256) * t2, tail = tiles - head, whole = tiles / 256 * 256;
          CHECK(head <= whole && head > whole - t2 && tail > 0 && tail <= 128);
          CHECK(S2 >= 2 && tail * S2 <= 256 && orion_wgrad_effective_splits(M, S2) == S2);
        } else {
          CHECK(S2 == 1);
        }
      }
  {  // Llama-7B gate_up weight gradient at 16k tokens: 80 tile rows unsplit + 6 rows at S2 = 2
    int S2 = 0;
    CHECK(orion_wgrad_tail_rows(16384, 22016, 4096, &S2) == 80 * 256 && S2 == 2);
    CHECK(orion_wgrad_tail_rows(16384, 12288, 4096, &S2) == 0);  // 768 tiles: whole rounds
    // GPT-2's LM head at 4k tokens: 170 tile rows unsplit, 26.5 rows at S2 = 3
    CHECK(orion_wgrad_tail_rows(4096, 50304, 768, &S2) == 170 * 256 && S2 == 3);
  }
  // scratch sizing is monotone and positive
  for (int rows = 1; rows < (1 << 20); rows = rows * 3 + 1) {
    CHECK(orion_layernorm_bwd_blocks(rows) >= 1 && orion_layernorm_bwd_blocks(rows) <= 1024);
    CHECK(orion_rmsnorm_bwd_blocks(rows) >= 1);
    CHECK(orion_colsum_scratch(rows, 768) >= 768);
  }
  // argument validation: every one of these must be rejected without a launch
  std::vector<uint16_t> buf(1 << 16);
  const void* p = buf.data();
  const void* mis = reinterpret_cast<const char*>(buf.data()) + 2;  // not 16-byte aligned
  void* o = buf.data();
  CHECK(orion_gemm(p, 64, p, 64, 64, 64, 48, 0, 0, o, 64, nullptr, nullptr, 0, nullptr, 0, 0) == -1);   // K % 64
  CHECK(orion_gemm(p, 64, p, 64, 64, 60, 64, 0, 0, o, 64, nullptr, nullptr, 0, nullptr, 0, 0) == -1);   // N % 8
  CHECK(orion_gemm(p, 66, p, 64, 64, 64, 64, 0, 0, o, 64, nullptr, nullptr, 0, nullptr, 0, 0) == -1);   // ld % 8
  CHECK(orion_gemm(mis, 64, p, 64, 64, 64, 64, 0, 0, o, 64, nullptr, nullptr, 0, nullptr, 0, 0) == -2); // alignment
  CHECK(orion_gemm(p, 64, p, 64, 64, 64, 64, 0, 1, o, 64, nullptr, nullptr, 0, nullptr, 0, 0) == -3);   // bias missing
  CHECK(orion_gemm(p, 64, p, 64, 64, 64, 64, 0, 2, o, 64, p, nullptr, 64, nullptr, 0, 0) == -3);        // gelu out2 missing
  CHECK(orion_gemm(p, 64, p, 64, 64, 64, 64, 1, 3, o, 64, nullptr, nullptr, 0, nullptr, 0, 0) == -3);   // pre missing
  CHECK(orion_gemm(p, 64, p, 64, 0, 64, 64, 0, 0, o, 64, nullptr, nullptr, 0, nullptr, 0, 0) == -1);    // M = 0
  CHECK(orion_gemm(p, 64, p, 64, 64, 64, 64, 0, 5, o, 128, nullptr, o, 128, p, 128, 0) == -3);         // swiglu: NN only
  CHECK(orion_gemm(p, 64, p, 64, 64, 64, 64, 1, 5, o, 128, nullptr, nullptr, 0, p, 128, 0) == -3);     // swiglu: out2 missing
  CHECK(orion_gemm(p, 64, p, 64, 64, 64, 64, 1, 5, o, 128, nullptr, o, 128, nullptr, 0, 0) == -3);     // swiglu: pre missing
  float part[4096];
  CHECK(orion_gemm(p, 64, p, 64, 64, 64, 64, 1, 0, o, 64, nullptr, nullptr, 0, nullptr, 0, 0, o, 0, part) == -3);  // db needs epi 3
  CHECK(orion_gemm(p, 64, p, 64, 64, 64, 64, 1, 3, o, 64, nullptr, nullptr, 0, p, 64, 0, o, 0, nullptr) == -3);  // db needs scratch
  CHECK(orion_gemm(p, 64, p, 64, 64, 64, 64, 1, 3, o, 72, nullptr, nullptr, 0, p, 64, 0, o, 0, part) == -3);     // db needs ldo == N
  CHECK(orion_gemm_colsum_scratch(65, 64) == (2 + 32) * 64);
  CHECK(orion_wgrad(p, 64, p, 64, 33, 64, 64, 1, nullptr, o, nullptr, 0, 0, 0, 0) == -1);              // M % BK
  CHECK(orion_wgrad(mis, 64, p, 64, 64, 64, 64, 1, nullptr, o, nullptr, 0, 0, 0, 0) == -2);            // alignment
  CHECK(orion_wgrad(p, 64, p, 64, 4096, 64, 64, 2, nullptr, o, nullptr, 0, 0, 0, 0) == -4);            // slabs missing
  if (failures) return 1;
  std::printf("host logic ok\n");
  return 0;
}
