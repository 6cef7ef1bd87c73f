// Forward and input-gradient GEMMs of the linear layers (gfx950): argument checks and the
// launch of the in-tree kernel, csrc/gemm16.hip (v_mfma_f32_16x16x32_bf16, persistent walk,
// fused epilogues).
//
//   forward  (NT):  Y[m][n]  = sum_k X[m][k] W[n][k]          W stored [N][K] (nn.Linear)
//   dgrad    (NN):  dX[m][n] = sum_k dY[m][k] W[k][n]         W stored [K][N] (same tensor)
//
// Epilogues (fp32, before the single bf16 rounding of the output):
//   EPI_STORE      out = acc
//   EPI_BIAS       out = acc + bias[n]                                       (QKV projection)
//   EPI_BIAS_GELU  out = a = acc + bias[n], out2 = gelu_tanh(a)              (MLP c_fc)
//   EPI_GELU_BWD   out = acc * gelu_tanh'(pre[m][n] [+ bias[n]]), optional   (MLP c_proj dgrad)
//                  per-64-row column sums of out (the fc bias gradient)
//   EPI_SWIGLU_BWD out = acc * up * silu'(gate), out2 = acc * silu(gate)     (Llama down_proj
//                  with gate = pre[m][n], up = pre[m][N + n]                   dgrad)
//   EPI_SWIGLU     out = [gate | up] = X [W_g; W_u]^T, out2 = silu(gate) up   (Llama gate_up)
// The last two remove the separate bias+GELU forward and GELU backward HBM passes over the
// (tokens x 4C) activation.
//
// Round 4 pruned the variants no default path selected (docs/PERFORMANCE.md, "Kernel
// variants removed"): the 32x32x16 phased kernel (gemm_phased.hip), this file's 2-stage and
// ping-pong kernels (ORION_GEMM_CFG 0-8) and the two-workgroups-per-CU short-K kernel that
// measured slower than gemm16 on every shape.  Shapes gemm16 cannot address (a 256-row band
// past the 32-bit buffer offsets) return -1 and the caller takes hipBLASLt.
#include <cstdlib>

#include "gemm_common.h"

using namespace orion;

int orion_colsum_partials2(const float* part, float* mid, void* out, int P, int C, int f32,
                           hipStream_t st);

// Diagnostic flags (GemmArgs::flags): 4 = gemm16's stamped instantiation (EPI_STORE, the
// stamp buffer passed as `pre`), 32 = with its stores waited for, 64 = one workgroup per work
// item instead of the persistent walk, bits 8-15 = the m-tile group size of the work order.
// Read once from ORION_GEMM_DIAG; scripts change them in-process through orion_gemm_set_diag
// (the gemm_diag op).
static int g_diag = -1;

static int gemm_diag() {
  if (g_diag < 0) {
    const char* e = getenv("ORION_GEMM_DIAG");
    g_diag = e ? atoi(e) : 0;
  }
  return g_diag;
}

// flags < 0: query only
int orion_gemm_set_diag(int flags) {
  const int old = gemm_diag();
  if (flags >= 0) g_diag = flags;
  return old;
}

// EPI_GELU_BWD with db: db[N] (fp32 when db_f32, else bf16) = column sums of the result (the
// bias gradient) through part (orion_gemm_colsum_scratch(M, N) floats): gemm16's per-64-row
// partials, folded by a second pass.
int orion_gemm_colsum_scratch(int M, int N) { return ((M + 63) / 64 + 32) * N; }

// out[M][N] = X[M][K] . op(W) with op(W) = W^T for W [N][K] (wkm = 0) or W for W [K][N]
// (wkm = 1), epilogue `epi` (GemmEpi).  Requirements (else -1): K % 64 == 0, N % 8 == 0,
// N >= 8, 8-element aligned leading dims, 16-byte aligned base pointers, 32-bit offsets
// within one 256-row band (gemm16_ok).
int orion_gemm(const void* X, long ldx, const void* W, long ldw, int M, int N, int K, int wkm,
               int epi, void* out, long ldo, const void* bias, void* out2, long ldo2,
               const void* pre, long ldp, hipStream_t st, void* db, int db_f32, float* part) {
  // epi | GEMM_DERIV: the GELU derivative form (GemmArgs::deriv) of EPI_BIAS_GELU / EPI_GELU_BWD
  const int deriv = (epi & GEMM_DERIV) ? 1 : 0;
  epi &= ~GEMM_DERIV;
  if (deriv && epi != EPI_BIAS_GELU && epi != EPI_GELU_BWD) return -3;
  if (deriv && epi == EPI_GELU_BWD && bias) return -3;  // the bias is inside the stored derivative
  if (M < 1 || K < 64 || K % 64 || N % 8 || N < 8) return -1;
  if ((ldx | ldw | ldo) % 8) return -1;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) |
       reinterpret_cast<uintptr_t>(out)) & 15) return -2;
  if ((epi == EPI_BIAS || epi == EPI_BIAS_GELU) && !bias) return -3;
  if (epi == EPI_BIAS_GELU && (!out2 || ldo2 % 8 || (reinterpret_cast<uintptr_t>(out2) & 15))) return -3;
  if ((epi == EPI_GELU_BWD || epi == EPI_SWIGLU_BWD) && (!pre || ldp % 8 || (reinterpret_cast<uintptr_t>(pre) & 15)))
    return -3;
  if (epi == EPI_SWIGLU_BWD && (!wkm || !out2 || ldo2 % 8 || (reinterpret_cast<uintptr_t>(out2) & 15))) return -3;
  if (db && (epi != EPI_GELU_BWD || !part || ldo != N)) return -3;
  GemmArgs a{(const bf16_t*)X, ldx, (const bf16_t*)W, ldw, (bf16_t*)out, ldo,
             (const bf16_t*)bias, (bf16_t*)out2, ldo2, (const bf16_t*)pre, ldp,
             M, N, K, (N + 255) / 256, gemm_diag()};
  a.deriv = deriv;
  if ((a.flags & 4) && epi <= EPI_BIAS_GELU) a.slabs = (float*)pre;  // slot stamps (diagnostic)
  if (!gemm16_ok(a, wkm)) return -1;
  const int rows = (M + 63) / 64;
  if (db) a.colsum = part;
  int rc = gemm16(a, wkm, epi, st);
  if (rc == 0 && db) rc = orion_colsum_partials2(part, part + (long)rows * N, db, rows, N, db_f32, st);
  return rc;
}

// LM head (csrc/lmhead.hip): the forward GEMM with the exp epilogue (epi = EPI_EXP, NT W
// [N][K]: row partial sums into rowpart[M][npart = ceil(N / 128)], the target logits into
// tlog) and the input-gradient GEMM with the per-row scale (epi = EPI_ROWSCALE, W [K][N]).
int orion_gemm_lm(const void* X, long ldx, const void* W, long ldw, int M, int N, int K, int epi,
                  void* out, long ldo, float* rowpart, const int64_t* tgt, float* tlog, const float* cref,
                  const float* rs, hipStream_t st) {
  if (M < 1 || K < 64 || K % 64 || N % 8 || N < 8) return -1;
  if ((ldx | ldw | ldo) % 8) return -1;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) |
       reinterpret_cast<uintptr_t>(out)) & 15) return -2;
  if (epi == EPI_EXP && (!rowpart || !tgt || !tlog || !cref)) return -3;
  if (epi == EPI_ROWSCALE && !rs) return -3;
  if (epi != EPI_EXP && epi != EPI_ROWSCALE) return -3;
  GemmArgs a{(const bf16_t*)X, ldx, (const bf16_t*)W, ldw, (bf16_t*)out, ldo,
             nullptr, nullptr, 0, nullptr, 0, M, N, K, (N + 255) / 256, gemm_diag()};
  a.rowpart = rowpart;
  a.npart = (N + 127) / 128;
  a.tgt = tgt;
  a.tlog = tlog;
  a.cref = cref;
  a.rs = rs;
  const int wkm = epi == EPI_ROWSCALE ? 1 : 0;
  if (!gemm16_ok(a, wkm)) return -1;
  return gemm16(a, wkm, epi, st);
}

// Llama's packed QKV projection with RoPE in the epilogue (EPI_ROPE, NT W [N][K]): columns
// [0, rcols) are heads of D = 128 rotated at position (m % T) + pos0 by the fp32 tables
// cosv / sinv [positions][D / 2]; the rest (v) are stored as computed.
int orion_gemm_rope(const void* X, long ldx, const void* W, long ldw, int M, int N, int K, void* out,
                    long ldo, const float* cosv, const float* sinv, int T, int pos0, int rcols, int D,
                    hipStream_t st) {
  if (M < 1 || K < 64 || K % 64 || N % 8 || N < 8) return -1;
  if ((ldx | ldw | ldo) % 8) return -1;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) |
       reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(cosv) |
       reinterpret_cast<uintptr_t>(sinv)) & 15) return -2;
  // a wave's 128 columns are one head (D = 128: Llama's head dim); the rotated range whole waves
  if (D != 128 || rcols % 128 || rcols > N || T < 1 || pos0 < 0 || !cosv || !sinv) return -3;
  GemmArgs a{(const bf16_t*)X, ldx, (const bf16_t*)W, ldw, (bf16_t*)out, ldo,
             nullptr, nullptr, 0, nullptr, 0, M, N, K, (N + 255) / 256, gemm_diag()};
  a.rcos = cosv;
  a.rsin = sinv;
  a.rT = T;
  a.rpos0 = pos0;
  a.rcols = rcols;
  a.rD = D;
  if (!gemm16_ok(a, 0)) return -1;
  return gemm16(a, 0, EPI_ROPE, st);
}

// Llama's gate_up projection with SwiGLU in the epilogue (EPI_SWIGLU, NT W = [W_gate; W_up]
// [2F][K]): gu [M][2F] (kept for the backward) and h = silu(gate) * up [M][F].  F % 128 == 0
// (a wave's 128 tile columns are 64 gate + 64 up features); the whole W within 32-bit offsets.
int orion_gemm_swiglu(const void* X, long ldx, const void* W, long ldw, int M, int F, int K, void* gu,
                      long ldg, void* h, long ldh, hipStream_t st) {
  if (M < 1 || K < 64 || K % 64 || F < 128 || F % 128) return -1;
  if ((ldx | ldw | ldg | ldh) % 8) return -1;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(gu) |
       reinterpret_cast<uintptr_t>(h)) & 15) return -2;
  const int N = 2 * F;
  if ((long)N * ldw * 2 >= 0xFFFFFF00L) return -1;
  GemmArgs a{(const bf16_t*)X, ldx, (const bf16_t*)W, ldw, (bf16_t*)gu, ldg,
             nullptr, (bf16_t*)h, ldh, nullptr, 0, M, N, K, N / 256, gemm_diag()};
  if (!gemm16_ok(a, 0)) return -1;
  return gemm16(a, 0, EPI_SWIGLU, st);
}
