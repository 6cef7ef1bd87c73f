// torch.ops.orion_amd.* registrations for the gfx950 kernels in csrc/*.hip.
//
// The kernels themselves are compiled without any torch headers; this file is
// the only place that sees at::Tensor.  Every op launches on the current
// PyTorch HIP stream (so ops compose with torch streams and HIP-graph capture)
// and allocates outputs through the PyTorch caching allocator.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <tuple>

#include "attn_params.h"

// launchers (csrc/*.hip)
int orion_layernorm_fwd(const void*, const void*, const void*, void*, float*, float*, int, int,
                        float, const void*, void*, const void*, hipStream_t,
                        const int64_t* idx = nullptr, int T = 0, long V = 0, int* err = nullptr);
int orion_embed_scatter_add(const void*, const int64_t*, float*, long, int, long, int*, hipStream_t);
int orion_batch_sum(const void*, void*, int, long, int, hipStream_t);
int orion_layernorm_bwd_blocks(int rows);
int orion_layernorm_bwd(const void*, const void*, const void*, const float*, const float*, void*,
                        void*, void*, float*, int, int, const void*, void*, int, hipStream_t);
int orion_colsum_bf16(const void*, void*, float*, int, int, int, hipStream_t);
int orion_bias_gelu_fwd(const void*, const void*, void*, long, int, hipStream_t);
int orion_bias_gelu_bwd(const void*, const void*, const void*, void*, float*, int, int, hipStream_t);
int orion_colsum_partials2(const float*, float*, void*, int, int, int, hipStream_t);
int orion_colsum_scratch(int rows, int C);
int orion_swiglu_fwd(const void*, void*, long, int, hipStream_t);
int orion_swiglu_bwd(const void*, const void*, void*, long, int, hipStream_t);
int orion_scale_bf16(void*, const float*, long, hipStream_t);
int orion_slab_sum(const float*, int, long, void*, const float*, int, int, hipStream_t);
int orion_wgrad_splits(int, int, int);
int orion_wgrad_effective_splits(int, int);
int orion_wgrad_tail_rows(int, int, int, int*);
int orion_wgrad(const void*, long, const void*, long, int, int, int, int, float*, void*,
                const float*, int, int, int, hipStream_t);
int orion_xent_fwd_bwd(void*, const int64_t*, float*, float*, float*, long, int, long, int*, hipStream_t);
int orion_sumsq_partials();
int orion_grad_sumsq(const void*, long, int, float*, float*, hipStream_t);
int orion_adamw_flat(void*, float*, float*, float*, const void*, int, const uint8_t*, const float*,
                     const float*, long, hipStream_t);
int orion_rmsnorm_fwd(const void*, const void*, void*, float*, int, int, float, const void*, void*,
                      hipStream_t);
int orion_rmsnorm_bwd_blocks(int rows);
int orion_rmsnorm_bwd(const void*, const void*, const void*, const float*, void*, void*, float*,
                      int, int, const void*, int, hipStream_t);
int orion_rope(const void*, long, long, long, void*, long, long, long, const float*, const float*,
               int, int, int, int, int, float, hipStream_t);
int orion_attn_fwd(const orion::AttnParams&, int, bool, hipStream_t);
int orion_attn_bwd(const orion::AttnParams&, int, bool, float*, hipStream_t);
int orion_attn_dq_convert(const float*, void*, long, long, long, int, int, int, int, hipStream_t);
int orion_attn_bwd_split(const orion::AttnParams&, int, bool, float*, hipStream_t);
int orion_gemm(const void*, long, const void*, long, int, int, int, int, int, void*, long,
               const void*, void*, long, const void*, long, hipStream_t, void* db = nullptr,
               int db_f32 = 0, float* part = nullptr);
int orion_gemm_colsum_scratch(int M, int N);
int orion_gemm_lm(const void*, long, const void*, long, int, int, int, int, void*, long, float*,
                  const int64_t*, float*, const float*, const float*, hipStream_t);
int orion_gemm_rope(const void*, long, const void*, long, int, int, int, void*, long, const float*, const float*,
                    int, int, int, int, hipStream_t);
int orion_gemm_swiglu(const void*, long, const void*, long, int, int, int, void*, long, void*, long, hipStream_t);
int orion_blaslt_linear_res(const void*, long, const void*, long, const void*, const void*, long, void*, long, int,
                            int, int, hipStream_t);
int orion_lmhead_fold(const float*, int, const float*, const int64_t*, long, float*, void*, long, int, long,
                      const void*, long, const void*, long, int, float*, float*, float*, int*, int*, float*,
                      float*, int*, hipStream_t);
int orion_lmhead_bwd_prep(const void*, long, int, long, const int64_t*, long, int, const float*, const float*,
                          const float*, float*, void*, int, hipStream_t);
int orion_gemm_set_diag(int flags);

namespace {

using at::Tensor;

hipStream_t cur_stream() {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
}

// one int per device, allocated on first use (before any graph capture: the first embedding
// call of a process runs eagerly), zeroed once
int* id_error_flag(int device) {
  static int* flags[64] = {nullptr};
  TORCH_CHECK(device >= 0 && device < 64, "device index out of range");
  if (!flags[device]) {
    int* p = nullptr;
    TORCH_CHECK(hipMalloc(&p, sizeof(int)) == hipSuccess && hipMemset(p, 0, sizeof(int)) == hipSuccess,
                "id_error_flag: allocation failed");
    flags[device] = p;
  }
  return flags[device];
}

void check_launch(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "orion_amd kernel launch failed: ", what, " (code ", rc, ")");
}

void check_bf16(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16, got ", t.scalar_type());
}

// a gradient output: bf16, or fp32 (the gradient arena's default dtype)
void check_grad_out(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat, name,
              " must be bfloat16 or float32, got ", t.scalar_type());
}

int is_f32(const Tensor& t) { return t.scalar_type() == at::kFloat ? 1 : 0; }

// an optional in-place output (a parameter's gradient-arena slice, ops/grad_sink.py): must be
// a contiguous bf16 or fp32 vector of n elements
bool has_out(const c10::optional<Tensor>& o, int64_t n, const char* name) {
  if (!o.has_value() || !o->defined()) return false;
  check_grad_out(*o, name);
  TORCH_CHECK(o->is_contiguous() && o->numel() == n, name, " must be contiguous with ", n,
              " elements, got ", o->sizes());
  return true;
}

// ------------------------------------------------------------------ layernorm
std::tuple<Tensor, Tensor, Tensor> layernorm_fwd(const Tensor& x, const Tensor& w,
                                                 const c10::optional<Tensor>& b, double eps) {
  check_bf16(x, "x");
  check_bf16(w, "weight");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto xc = x.contiguous();
  const int C = x.size(-1);
  const int rows = x.numel() / C;
  auto y = at::empty_like(xc);
  auto opts = x.options().dtype(at::kFloat);
  auto mean = at::empty({rows}, opts), rstd = at::empty({rows}, opts);
  const void* bp = nullptr;
  Tensor bc;
  if (b.has_value() && b->defined()) {
    check_bf16(*b, "bias");
    bc = b->contiguous();
    bp = bc.data_ptr();
  }
  check_launch(orion_layernorm_fwd(xc.data_ptr(), w.contiguous().data_ptr(), bp, y.data_ptr(),
                                   mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, C,
                                   (float)eps, nullptr, nullptr, nullptr, cur_stream()),
               "layernorm_fwd");
  return {y, mean, rstd};
}

// s = x + r ; y = LayerNorm(s)  -> (s, y, mean, rstd)
std::tuple<Tensor, Tensor, Tensor, Tensor> add_layernorm_fwd(const Tensor& x, const Tensor& r,
                                                             const Tensor& w,
                                                             const c10::optional<Tensor>& b,
                                                             double eps,
                                                             const c10::optional<Tensor>& rbias) {
  check_bf16(x, "x");
  check_bf16(r, "residual");
  check_bf16(w, "weight");
  TORCH_CHECK(x.sizes() == r.sizes(), "add_layernorm: shape mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto xc = x.contiguous(), rc = r.contiguous();
  const int C = x.size(-1);
  const int rows = x.numel() / C;
  auto y = at::empty_like(xc), sum = at::empty_like(xc);
  auto opts = x.options().dtype(at::kFloat);
  auto mean = at::empty({rows}, opts), rstd = at::empty({rows}, opts);
  const void* bp = nullptr;
  Tensor bc, rbc;
  if (b.has_value() && b->defined()) {
    check_bf16(*b, "bias");
    bc = b->contiguous();
    bp = bc.data_ptr();
  }
  if (rbias.has_value() && rbias->defined()) {
    check_bf16(*rbias, "branch bias");
    rbc = rbias->contiguous();
  }
  check_launch(orion_layernorm_fwd(xc.data_ptr(), w.contiguous().data_ptr(), bp, y.data_ptr(),
                                   mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, C,
                                   (float)eps, rc.data_ptr(), sum.data_ptr(),
                                   rbc.defined() ? rbc.data_ptr() : nullptr, cur_stream()),
               "add_layernorm_fwd");
  return {sum, y, mean, rstd};
}

// s = wte[idx] + wpe[t] ; y = LayerNorm(s)  -> (s, y, mean, rstd); idx (B, T) int64
std::tuple<Tensor, Tensor, Tensor, Tensor> embed_layernorm_fwd(const Tensor& idx, const Tensor& wte,
                                                               const Tensor& wpe, const Tensor& w,
                                                               const c10::optional<Tensor>& b,
                                                               double eps) {
  check_bf16(wte, "wte");
  check_bf16(wpe, "wpe");
  check_bf16(w, "weight");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kLong && idx.dim() == 2,
              "embed_layernorm: idx must be a (B, T) int64 GPU tensor");
  TORCH_CHECK(wte.dim() == 2 && wpe.dim() == 2 && wte.size(1) == wpe.size(1),
              "embed_layernorm: wte (V, C) and wpe (Tmax, C) must share C");
  const int T = idx.size(1);
  TORCH_CHECK(T <= wpe.size(0), "embed_layernorm: sequence longer than the position table");
  c10::hip::HIPGuardMasqueradingAsCUDA g(wte.device());
  auto ic = idx.contiguous();
  const int C = wte.size(1);
  const int rows = ic.numel();
  auto opts = wte.options();
  auto y = at::empty({idx.size(0), T, C}, opts), sum = at::empty({idx.size(0), T, C}, opts);
  auto fopts = opts.dtype(at::kFloat);
  auto mean = at::empty({rows}, fopts), rstd = at::empty({rows}, fopts);
  const void* bp = nullptr;
  Tensor bc;
  if (b.has_value() && b->defined()) {
    check_bf16(*b, "bias");
    bc = b->contiguous();
    bp = bc.data_ptr();
  }
  auto wtec = wte.contiguous(), wpec = wpe.contiguous();
  check_launch(orion_layernorm_fwd(wtec.data_ptr(), w.contiguous().data_ptr(), bp, y.data_ptr(),
                                   mean.data_ptr<float>(), rstd.data_ptr<float>(), rows, C,
                                   (float)eps, wpec.data_ptr(), sum.data_ptr(), nullptr,
                                   cur_stream(), ic.data_ptr<int64_t>(), T, wte.size(0),
                                   id_error_flag(wte.device().index())),
               "embed_layernorm_fwd");
  return {sum, y, mean, rstd};
}

// out[idx[i]] += dx[i] (fp32 atomics); out: the (V, C) fp32 table gradient
void embed_scatter_add_(const Tensor& dx, const Tensor& idx, Tensor out) {
  check_bf16(dx, "dx");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kLong, "idx must be int64 on the GPU");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.dim() == 2,
              "out must be a contiguous (V, C) float32 GPU tensor");
  const int C = out.size(1);
  TORCH_CHECK(dx.numel() == idx.numel() * C, "embed_scatter_add: dx must be (N, C) for N ids");
  c10::hip::HIPGuardMasqueradingAsCUDA g(dx.device());
  auto dxc = dx.contiguous(), ic = idx.contiguous();
  check_launch(orion_embed_scatter_add(dxc.data_ptr(), ic.data_ptr<int64_t>(), out.data_ptr<float>(),
                                       ic.numel(), C, out.size(0),
                                       id_error_flag(dx.device().index()), cur_stream()),
               "embed_scatter_add_");
}

// Token-id error flag of a device: nonzero once an embedding kernel saw an id outside its
// table (the id was clamped / skipped, nothing outside the table was touched).  Reads the
// flag (synchronises the current stream) and clears it.
int64_t embed_id_error(int64_t device) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, (int)device));
  int* f = id_error_flag((int)device);
  int v = 0;
  auto st = cur_stream();
  TORCH_CHECK(hipMemcpyAsync(&v, f, sizeof(int), hipMemcpyDeviceToHost, st) == hipSuccess &&
                  hipMemsetAsync(f, 0, sizeof(int), st) == hipSuccess &&
                  hipStreamSynchronize(st) == hipSuccess,
              "embed_id_error: flag read failed");
  return v;
}

// out (n) = sum over the leading dim of x (B, ...): fp32 or bf16 out (a gradient-arena slice)
void batch_sum_(const Tensor& x, Tensor out) {
  check_bf16(x, "x");
  const long n = x.numel() / x.size(0);
  TORCH_CHECK(has_out(out, n, "out"), "batch_sum_: out required");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto xc = x.contiguous();
  check_launch(orion_batch_sum(xc.data_ptr(), out.data_ptr(), x.size(0), n, is_f32(out), cur_stream()),
               "batch_sum_");
}

std::tuple<Tensor, Tensor, Tensor, Tensor> layernorm_bwd(const Tensor& dy, const Tensor& x,
                                                         const Tensor& w, const Tensor& mean,
                                                         const Tensor& rstd, bool has_bias,
                                                         const c10::optional<Tensor>& dres,
                                                         bool want_dx_colsum,
                                                         const c10::optional<Tensor>& dw_out,
                                                         const c10::optional<Tensor>& db_out,
                                                         const c10::optional<Tensor>& dxs_out) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto dyc = dy.contiguous(), xc = x.contiguous();
  const int C = x.size(-1);
  const int rows = x.numel() / C;
  auto dx = at::empty_like(xc);
  // a given *_out (a parameter's gradient-arena slice, ops/grad_sink.py) is written in place
  // and its return slot is left undefined
  const bool w_in = has_out(dw_out, C, "dw_out"), b_in = has_bias && has_out(db_out, C, "db_out");
  const bool s_in = want_dx_colsum && has_out(dxs_out, C, "dxs_out");
  // one output dtype for the three column sums: fp32 if any given slice is fp32 (the caller
  // converts returned gradients to the parameter dtype)
  int f32 = 0;
  for (auto* o : {&dw_out, &db_out, &dxs_out})
    if (o->has_value() && (*o)->defined()) f32 |= is_f32(**o);
  for (auto* o : {&dw_out, &db_out, &dxs_out})
    if (o->has_value() && (*o)->defined())
      TORCH_CHECK(is_f32(**o) == f32, "layernorm_bwd: gradient outputs must share one dtype");
  auto gopts = f32 ? w.options().dtype(at::kFloat) : w.options();
  Tensor dw = w_in ? *dw_out : at::empty({C}, gopts);
  Tensor db = has_bias ? (b_in ? *db_out : at::empty({C}, gopts)) : Tensor();
  const int nb = orion_layernorm_bwd_blocks(rows);
  auto part = at::empty({3 * (long)nb * C + 48L * C}, x.options().dtype(at::kFloat));
  Tensor dxs = want_dx_colsum ? (s_in ? *dxs_out : at::empty({C}, f32 ? gopts : x.options())) : Tensor();
  Tensor drc;
  if (dres.has_value() && dres->defined()) {
    check_bf16(*dres, "dres");
    drc = dres->contiguous();
  }
  check_launch(orion_layernorm_bwd(dyc.data_ptr(), xc.data_ptr(), w.contiguous().data_ptr(),
                                   mean.data_ptr<float>(), rstd.data_ptr<float>(), dx.data_ptr(),
                                   dw.data_ptr(), has_bias ? db.data_ptr() : nullptr,
                                   part.data_ptr<float>(), rows, C, drc.defined() ? drc.data_ptr() : nullptr,
                                   want_dx_colsum ? dxs.data_ptr() : nullptr, f32, cur_stream()),
               "layernorm_bwd");
  return {dx, w_in ? Tensor() : dw, b_in ? Tensor() : db, s_in ? Tensor() : dxs};
}

// ------------------------------------------------------------------ activations
Tensor bias_gelu_fwd(const Tensor& x, const c10::optional<Tensor>& b) {
  check_bf16(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto xc = x.contiguous();
  auto y = at::empty_like(xc);
  const int C = x.size(-1);
  Tensor bc;
  const void* bp = nullptr;
  if (b.has_value() && b->defined()) {
    check_bf16(*b, "bias");
    bc = b->contiguous();
    bp = bc.data_ptr();
  }
  check_launch(orion_bias_gelu_fwd(xc.data_ptr(), bp, y.data_ptr(), xc.numel(), C, cur_stream()),
               "bias_gelu_fwd");
  return y;
}

std::tuple<Tensor, Tensor> bias_gelu_bwd(const Tensor& dy, const Tensor& x,
                                         const c10::optional<Tensor>& b,
                                         const c10::optional<Tensor>& db_out) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto dyc = dy.contiguous(), xc = x.contiguous();
  const int C = x.size(-1);
  const int rows = x.numel() / C;
  auto dx = at::empty_like(xc);
  Tensor db, bc;
  const void* bp = nullptr;
  float* part = nullptr;
  Tensor partt;
  if (b.has_value() && b->defined()) {
    bc = b->contiguous();
    bp = bc.data_ptr();
    db = has_out(db_out, C, "db_out") ? *db_out : at::empty({C}, b->options());
    partt = at::empty({(long)orion_colsum_scratch(rows, C)}, x.options().dtype(at::kFloat));
    part = partt.data_ptr<float>();
  }
  check_launch(orion_bias_gelu_bwd(dyc.data_ptr(), xc.data_ptr(), bp, dx.data_ptr(), part, rows,
                                   C, cur_stream()),
               "bias_gelu_bwd");
  if (part) {
    const int nb = orion_layernorm_bwd_blocks(rows);
    check_launch(orion_colsum_partials2(part, part + (long)nb * C, db.data_ptr(), nb, C,
                                        is_f32(db), cur_stream()),
                 "colsum");
  }
  return {dx, (db.defined() && has_out(db_out, C, "db_out")) ? Tensor() : db};
}

Tensor colsum(const Tensor& m, const c10::optional<Tensor>& out_) {
  check_bf16(m, "m");
  c10::hip::HIPGuardMasqueradingAsCUDA g(m.device());
  auto mc = m.contiguous();
  const int C = m.size(-1);
  const int rows = m.numel() / C;
  const bool given = has_out(out_, C, "out");
  auto out = given ? *out_ : at::empty({C}, m.options());
  auto part = at::empty({(long)orion_colsum_scratch(rows, C)}, m.options().dtype(at::kFloat));
  check_launch(orion_colsum_bf16(mc.data_ptr(), out.data_ptr(), part.data_ptr<float>(), rows, C,
                                 is_f32(out), cur_stream()),
               "colsum");
  return out;
}

Tensor swiglu_fwd(const Tensor& gu) {
  check_bf16(gu, "gate_up");
  c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
  auto c = gu.contiguous();
  const int F = gu.size(-1) / 2;
  const long rows = gu.numel() / (2L * F);
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  auto y = at::empty(sizes, gu.options());
  check_launch(orion_swiglu_fwd(c.data_ptr(), y.data_ptr(), rows, F, cur_stream()), "swiglu_fwd");
  return y;
}

Tensor swiglu_bwd(const Tensor& dy, const Tensor& gu) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(gu.device());
  auto c = gu.contiguous(), d = dy.contiguous();
  const int F = gu.size(-1) / 2;
  const long rows = gu.numel() / (2L * F);
  auto dgu = at::empty_like(c);
  check_launch(orion_swiglu_bwd(d.data_ptr(), c.data_ptr(), dgu.data_ptr(), rows, F, cur_stream()),
               "swiglu_bwd");
  return dgu;
}

void scale_(Tensor x, const Tensor& s) {
  check_bf16(x, "x");
  TORCH_CHECK(x.is_contiguous(), "scale_: x must be contiguous");
  TORCH_CHECK(s.scalar_type() == at::kFloat && s.numel() == 1, "scale must be one fp32 element");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_launch(orion_scale_bf16(x.data_ptr(), s.data_ptr<float>(), x.numel(), cur_stream()), "scale_");
}

// ------------------------------------------------------------------ cross entropy
// logits (N, V) bf16 contiguous -> overwritten with dlogits/n_valid; returns fp32 loss (scalar)
// LM head + cross-entropy without the logits pass (csrc/lmhead.hip): x (N, C), w (V, C) bf16,
// targets (N,) int64, cref a one-element fp32 device tensor (the running exp reference, updated
// in place).  Returns the mean loss, E' (N, V) bf16 (exp(logit - ref) with the one-hot term
// folded in), invz (N,) = 1 / Z per row and inv_n (1,) = 1 / n_valid.
std::tuple<Tensor, Tensor, Tensor, Tensor> lmhead_fwd(const Tensor& x, const Tensor& w, const Tensor& targets,
                                                      int64_t ignore_index, Tensor cref) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "lmhead_fwd: x must be (N, C) with unit column stride");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && w.size(1) == x.size(1), "lmhead_fwd: w must be a contiguous (V, C)");
  TORCH_CHECK(targets.scalar_type() == at::kLong && targets.numel() == x.size(0), "lmhead_fwd: targets (N,) int64");
  TORCH_CHECK(cref.scalar_type() == at::kFloat && cref.numel() == 1 && cref.is_cuda(), "lmhead_fwd: cref fp32 (1,)");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  const long N = x.size(0);
  const int Cd = (int)x.size(1), V = (int)w.size(0);
  TORCH_CHECK(N < (1L << 31) && V % 8 == 0 && Cd % 64 == 0, "lmhead_fwd: unsupported shape");
  auto t = targets.contiguous();
  auto fopts = x.options().dtype(at::kFloat);
  auto E = at::empty({N, (long)V}, x.options());
  const int npart = (V + 127) / 128;
  auto part = at::empty({N * npart}, fopts);
  auto tlog = at::empty({N}, fopts);
  auto invz = at::empty({N}, fopts);
  auto lse = at::empty({N}, fopts);
  auto lrow = at::empty({N}, fopts);
  auto ints = at::empty({4 + N}, x.options().dtype(at::kInt));
  auto loss = at::empty({}, fopts);
  auto inv_n = at::empty({1}, fopts);
  check_launch(orion_gemm_lm(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), (int)N, V, Cd, 6, E.data_ptr(),
                             V, part.data_ptr<float>(), t.data_ptr<int64_t>(), tlog.data_ptr<float>(),
                             cref.data_ptr<float>(), nullptr, cur_stream()),
               "lmhead_fwd gemm");
  check_launch(orion_lmhead_fold(part.data_ptr<float>(), npart, tlog.data_ptr<float>(), t.data_ptr<int64_t>(),
                                 ignore_index, cref.data_ptr<float>(), E.data_ptr(), V, V, N, x.data_ptr(),
                                 x.stride(0), w.data_ptr(), w.stride(0), Cd, invz.data_ptr<float>(),
                                 lse.data_ptr<float>(), lrow.data_ptr<float>(), ints.data_ptr<int>(),
                                 ints.data_ptr<int>() + 4, loss.data_ptr<float>(), inv_n.data_ptr<float>(),
                                 id_error_flag(x.device().index()), cur_stream()),
               "lmhead_fold");
  return {loss, E, invz, inv_n};
}

// Backward prologue: srow (N,) fp32 = g / (Z n_valid) on valid rows, xs (N, C) = srow (.) x
// (transposed: xs is returned as (C, N), for the NT weight-gradient operand; N % 64 == 0 and
// C % 64 == 0).
std::tuple<Tensor, Tensor> lmhead_bwd_prep(const Tensor& x, const Tensor& targets, int64_t ignore_index,
                                           int64_t V, const Tensor& invz, const Tensor& inv_n, const Tensor& g,
                                           bool transposed) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "lmhead_bwd_prep: x (N, C)");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(x.device());
  const long N = x.size(0);
  const int Cd = (int)x.size(1);
  auto t = targets.contiguous();
  auto srow = at::empty({N}, x.options().dtype(at::kFloat));
  TORCH_CHECK(!transposed || (N % 64 == 0 && Cd % 64 == 0), "lmhead_bwd_prep: transposed needs N, C % 64 == 0");
  auto xs = transposed ? at::empty({(long)Cd, N}, x.options()) : at::empty({N, (long)Cd}, x.options());
  auto gf = g.to(at::kFloat).reshape({1}).contiguous();
  check_launch(orion_lmhead_bwd_prep(x.data_ptr(), x.stride(0), Cd, N, t.data_ptr<int64_t>(), ignore_index, (int)V,
                                     invz.data_ptr<float>(), inv_n.data_ptr<float>(), gf.data_ptr<float>(),
                                     srow.data_ptr<float>(), xs.data_ptr(), transposed ? 1 : 0, cur_stream()),
               "lmhead_bwd_prep");
  return {srow, xs};
}

// qkv (M, N) = x w^T with RoPE on the first rope_cols columns (heads of D; x (M, K) rows of
// T tokens each, position t + pos0): Llama's packed QKV projection (csrc/gemm16.hip EPI_ROPE).
Tensor gemm_rope(const Tensor& x, const Tensor& w, const Tensor& cos, const Tensor& sin, int64_t pos0, int64_t T,
                 int64_t rope_cols, int64_t D) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && x.stride(-1) == 1 && x.size(-1) == w.size(1),
              "gemm_rope: x (..., K) with unit stride, w contiguous (N, K)");
  TORCH_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
                  sin.is_contiguous() && cos.dim() == 2 && cos.size(1) == D / 2 && sin.sizes() == cos.sizes(),
              "gemm_rope: cos / sin fp32 contiguous (positions, D / 2)");
  const int64_t K = x.size(-1), N = w.size(0);
  auto x2 = x.reshape({-1, K});
  const int64_t M = x2.size(0);
  TORCH_CHECK(M % T == 0 && pos0 >= 0 && T + pos0 <= cos.size(0), "gemm_rope: rows must be whole sequences within the tables");
  TORCH_CHECK(M < (1LL << 31) && N < (1 << 30), "gemm_rope: shape too large");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  auto out = at::empty(sizes, x.options());
  check_launch(orion_gemm_rope(x2.data_ptr(), x2.stride(0), w.data_ptr(), w.stride(0), (int)M, (int)N, (int)K,
                               out.data_ptr(), N, cos.data_ptr<float>(), sin.data_ptr<float>(), (int)T, (int)pos0,
                               (int)rope_cols, (int)D, cur_stream()),
               "gemm_rope");
  return out;
}

// s (M, N) = x w^T (+ bias) (+ r): a branch's output projection with the residual add (hipBLASLt, the
// bias and r in its epilogue; csrc/blaslt.cpp).  x (M, K) and r (M, N) with unit column stride.
Tensor linear_residual(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias_in,
                       const c10::optional<Tensor>& r_in) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  const bool hb = bias_in.has_value() && bias_in->defined(), hr = r_in.has_value() && r_in->defined();
  if (hb) check_bf16(*bias_in, "bias");
  if (hr) check_bf16(*r_in, "r");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.stride(1) == 1 && w.is_contiguous() && x.size(1) == w.size(1) &&
                  (!hb || (bias_in->is_contiguous() && bias_in->numel() == w.size(0))) &&
                  (!hr || (r_in->dim() == 2 && r_in->stride(1) == 1 && r_in->size(0) == x.size(0) &&
                           r_in->size(1) == w.size(0))),
              "linear_residual: x (M, K), w (N, K), bias (N) or None, r (M, N) or None");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  auto out = at::empty({M, N}, x.options());
  check_launch(orion_blaslt_linear_res(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0),
                                       hb ? bias_in->data_ptr() : nullptr, hr ? r_in->data_ptr() : nullptr,
                                       hr ? r_in->stride(0) : N, out.data_ptr(), N, (int)M, (int)N, (int)K,
                                       cur_stream()),
               "linear_residual");
  return out;
}

// (gu (M, 2F), h (M, F)) = (x w^T, silu(gate) * up) for w = [W_gate; W_up] (2F, K): Llama's
// gate_up projection with the SwiGLU forward in the epilogue (csrc/gemm16.hip EPI_SWIGLU).
std::vector<Tensor> gemm_swiglu(const Tensor& x, const Tensor& w) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && x.dim() == 2 && x.stride(1) == 1 && x.size(1) == w.size(1),
              "gemm_swiglu: x (M, K) with unit stride, w contiguous (2F, K)");
  const int64_t M = x.size(0), K = x.size(1), F = w.size(0) / 2;
  TORCH_CHECK(w.size(0) % 256 == 0 && M < (1LL << 31) && F < (1 << 29), "gemm_swiglu: 2F % 256 == 0");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto gu = at::empty({M, 2 * F}, x.options());
  auto h = at::empty({M, F}, x.options());
  check_launch(orion_gemm_swiglu(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), (int)M, (int)F, (int)K,
                                 gu.data_ptr(), 2 * F, h.data_ptr(), F, cur_stream()),
               "gemm_swiglu");
  return {gu, h};
}

// dx (N, C) = srow (.) (e . w): the LM head's input gradient from E' (N, V) and w (V, C).
Tensor gemm_rowscale(const Tensor& e, const Tensor& w, const Tensor& srow) {
  check_bf16(e, "e");
  check_bf16(w, "w");
  TORCH_CHECK(e.dim() == 2 && e.stride(1) == 1 && w.dim() == 2 && w.is_contiguous() && w.size(0) == e.size(1),
              "gemm_rowscale: e (N, V), w (V, C)");
  c10::hip::HIPGuardMasqueradingAsCUDA g(e.device());
  const long N = e.size(0);
  const int V = (int)e.size(1), Cd = (int)w.size(1);
  auto out = at::empty({N, (long)Cd}, e.options());
  check_launch(orion_gemm_lm(e.data_ptr(), e.stride(0), w.data_ptr(), w.stride(0), (int)N, Cd, V, 7, out.data_ptr(),
                             Cd, nullptr, nullptr, nullptr, nullptr, srow.data_ptr<float>(), cur_stream()),
               "gemm_rowscale");
  return out;
}

Tensor xent_fwd_bwd(Tensor logits, const Tensor& targets, int64_t ignore_index) {
  check_bf16(logits, "logits");
  TORCH_CHECK(logits.is_contiguous() && logits.dim() == 2, "logits must be contiguous (N, V)");
  TORCH_CHECK(targets.scalar_type() == at::kLong, "targets must be int64");
  c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  const long N = logits.size(0);
  const int V = logits.size(1);
  auto t = targets.contiguous();
  auto fopts = logits.options().dtype(at::kFloat);
  auto losses = at::empty({N}, fopts);
  auto inv_n = at::empty({1}, fopts);
  auto loss = at::empty({}, fopts);
  check_launch(orion_xent_fwd_bwd(logits.data_ptr(), t.data_ptr<int64_t>(), losses.data_ptr<float>(),
                                  inv_n.data_ptr<float>(), loss.data_ptr<float>(), N, V,
                                  ignore_index, id_error_flag(logits.device().index()), cur_stream()),
               "xent_fwd_bwd");
  return loss;
}

// split-K combine: slabs (S, ...) fp32 -> bf16 sum over S, optionally times a device scalar
Tensor slab_sum(const Tensor& slabs, const c10::optional<Tensor>& scale) {
  TORCH_CHECK(slabs.scalar_type() == at::kFloat && slabs.is_contiguous() && slabs.dim() >= 2,
              "slab_sum: slabs must be contiguous fp32 (S, ...)");
  c10::hip::HIPGuardMasqueradingAsCUDA g(slabs.device());
  const int S = slabs.size(0);
  auto out = at::empty(slabs.sizes().slice(1), slabs.options().dtype(at::kBFloat16));
  const float* sc = nullptr;
  if (scale.has_value() && scale->defined()) {
    TORCH_CHECK(scale->scalar_type() == at::kFloat && scale->numel() == 1, "scale must be one fp32");
    sc = scale->data_ptr<float>();
  }
  check_launch(orion_slab_sum(slabs.data_ptr<float>(), S, out.numel(), out.data_ptr(), sc, 0, 0,
                              cur_stream()),
               "slab_sum");
  return out;
}

// dW = dy^T x over the token dim (csrc/wgrad.hip) into out (N1, N2) contiguous fp32 (the
// gradient arena) or bf16: overwritten, or added to when accumulate (micro-batch
// accumulation / tied weights).  splits = 0 picks the split-K count.
void wgrad_into(const Tensor& dy, const Tensor& x_in, const c10::optional<Tensor>& scale, Tensor out,
                bool accumulate, int64_t splits) {
  check_bf16(dy, "dy");
  check_bf16(x_in, "x");
  check_grad_out(out, "out");
  TORCH_CHECK(dy.dim() == 2 && x_in.dim() == 2 && dy.size(0) == x_in.size(0), "wgrad: dy (M,N1), x (M,N2)");
  const int M = dy.size(0), N1 = dy.size(1), N2 = x_in.size(1);
  // x given as the transposed view of a row-major (N2, M) tensor: the NT-operand kernel
  const bool xt = x_in.stride(0) == 1 && x_in.stride(1) != 1 && M % 64 == 0 && x_in.stride(1) % 8 == 0;
  const Tensor x = (xt || x_in.stride(1) == 1) ? x_in : x_in.contiguous();
  TORCH_CHECK(dy.stride(1) == 1, "wgrad: dy rows must be contiguous");
  const long ldx = xt ? x.stride(1) : x.stride(0);
  TORCH_CHECK(out.is_contiguous() && out.numel() == (int64_t)N1 * N2, "wgrad: out must be contiguous (N1, N2)");
  c10::hip::HIPGuardMasqueradingAsCUDA g(dy.device());
  int S = splits > 0 ? orion_wgrad_effective_splits(M, (int)splits) : orion_wgrad_splits(M, N1, N2);
  const float* sc = nullptr;
  if (scale.has_value() && scale->defined()) {
    TORCH_CHECK(scale->scalar_type() == at::kFloat && scale->numel() == 1, "scale must be one fp32");
    sc = scale->data_ptr<float>();
  }
  int S2 = 1;
  const int R1 = splits > 0 ? 0 : orion_wgrad_tail_rows(M, N1, N2, &S2);
  if (R1 > 0) {  // whole rounds unsplit, the tail rows split-K (orion_wgrad_tail_rows)
    check_launch(orion_wgrad(dy.data_ptr(), dy.stride(0), x.data_ptr(), ldx, M, R1, N2, 1,
                             nullptr, out.data_ptr(), sc, accumulate ? 1 : 0, is_f32(out),
                             xt ? 1 : 0, cur_stream()), "wgrad head");
    const int N1t = N1 - R1;
    auto slabs = at::empty({S2, N1t, N2}, dy.options().dtype(at::kFloat));
    const auto* dyt = static_cast<const char*>(dy.data_ptr()) + (size_t)R1 * dy.element_size();
    auto* outt = static_cast<char*>(out.data_ptr()) + (size_t)R1 * N2 * out.element_size();
    check_launch(orion_wgrad(dyt, dy.stride(0), x.data_ptr(), ldx, M, N1t, N2, S2,
                             slabs.data_ptr<float>(), nullptr, nullptr, 0, 0, xt ? 1 : 0, cur_stream()), "wgrad tail");
    check_launch(orion_slab_sum(slabs.data_ptr<float>(), S2, (long)N1t * N2, outt, sc,
                                accumulate ? 1 : 0, is_f32(out), cur_stream()), "wgrad tail slab_sum");
  } else if (S > 1) {
    auto slabs = at::empty({S, N1, N2}, dy.options().dtype(at::kFloat));
    check_launch(orion_wgrad(dy.data_ptr(), dy.stride(0), x.data_ptr(), ldx, M, N1, N2, S,
                             slabs.data_ptr<float>(), nullptr, nullptr, 0, 0, xt ? 1 : 0, cur_stream()), "wgrad");
    check_launch(orion_slab_sum(slabs.data_ptr<float>(), S, out.numel(), out.data_ptr(), sc,
                                accumulate ? 1 : 0, is_f32(out), cur_stream()), "wgrad slab_sum");
  } else {
    check_launch(orion_wgrad(dy.data_ptr(), dy.stride(0), x.data_ptr(), ldx, M, N1, N2, 1,
                             nullptr, out.data_ptr(), sc, accumulate ? 1 : 0, is_f32(out),
                             xt ? 1 : 0, cur_stream()), "wgrad");
  }
}

Tensor wgrad(const Tensor& dy, const Tensor& x, const c10::optional<Tensor>& scale, int64_t splits) {
  auto out = at::empty({dy.size(1), x.size(1)}, dy.options());
  wgrad_into(dy, x, scale, out, false, splits);
  return out;
}

int64_t wgrad_splits(int64_t M, int64_t N1, int64_t N2) { return orion_wgrad_splits(M, N1, N2); }
std::tuple<int64_t, int64_t> wgrad_tail_rows(int64_t M, int64_t N1, int64_t N2) {
  int s2 = 1;
  const int r1 = orion_wgrad_tail_rows((int)M, (int)N1, (int)N2, &s2);
  return {r1, s2};
}

// csrc/gemm.hip's diagnostic flags (stamps, one workgroup per work item): set in-process by
// the benchmark / timeline scripts; returns the previous value
int64_t gemm_diag(int64_t flags) { return orion_gemm_set_diag((int)flags); }

// ------------------------------------------------------------------ GEMM (csrc/gemm.hip)
// out (..., N) = x (..., K) . op(w) with op(w) = w^T for w (N, K) [w_kmajor = false, the
// nn.Linear forward] or w for w (K, N) [w_kmajor = true, the input gradient], and a fused
// epilogue: 0 store, 1 + bias, 2 + bias then GELU (returns (a, gelu(a))), 3 times
// GELU'(pre); 2 | 0x100 returns (GELU'(a), gelu(a)) (the derivative for gemm_gelu_bwd's
// pre_is_deriv form).  Returns (out, out2); out2 is undefined unless epi is 2.
std::tuple<Tensor, Tensor> gemm(const Tensor& x, const Tensor& w, bool w_kmajor, int64_t epi_in,
                                const c10::optional<Tensor>& bias, const c10::optional<Tensor>& pre) {
  TORCH_CHECK(epi_in == 0x102 || (epi_in >= 0 && epi_in <= 3), "gemm: unknown epilogue ", epi_in);
  const int64_t epi = epi_in & 0xFF;
  check_bf16(x, "x");
  check_bf16(w, "w");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "gemm: w must be a contiguous 2-D tensor");
  TORCH_CHECK(x.stride(-1) == 1, "gemm: x rows must be contiguous");
  const int64_t K = x.size(-1);
  TORCH_CHECK(K == (w_kmajor ? w.size(0) : w.size(1)), "gemm: reduction dims differ");
  const int64_t N = w_kmajor ? w.size(1) : w.size(0);
  auto x2 = x.reshape({-1, K});
  TORCH_CHECK(x2.stride(1) == 1, "gemm: x must flatten to rows");
  const int64_t M = x2.size(0);
  TORCH_CHECK(M < (1LL << 31) && N < (1 << 30), "gemm: shape too large");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  auto out = at::empty(sizes, x.options());
  Tensor out2, bc, pc;
  const void* bp = nullptr;
  const void* pp = nullptr;
  long ldp = 0;
  if (epi == 1 || epi == 2) {
    TORCH_CHECK(bias.has_value() && bias->defined(), "gemm: epilogue needs a bias");
    check_bf16(*bias, "bias");
    bc = bias->contiguous();
    TORCH_CHECK(bc.numel() == N, "gemm: bias must have N elements");
    bp = bc.data_ptr();
  }
  if (epi == 2) out2 = at::empty(sizes, x.options());
  if (epi <= 2 && pre.has_value() && pre->defined() && pre->nbytes() >= 8 * 8 * 1024)
    pp = pre->data_ptr();  // diagnostic: the gemm_diag(4) slot-stamp buffer (scripts/gemm16_stamps.py)
  if (epi == 3) {
    TORCH_CHECK(pre.has_value() && pre->defined(), "gemm: GELU backward needs the pre-activation");
    check_bf16(*pre, "pre");
    pc = pre->reshape({-1, N});
    TORCH_CHECK(pc.size(0) == M && pc.stride(1) == 1, "gemm: pre must be (M, N) with unit column stride");
    pp = pc.data_ptr();
    ldp = pc.stride(0);
  }
  check_launch(orion_gemm(x2.data_ptr(), x2.stride(0), w.data_ptr(), w.stride(0), (int)M, (int)N,
                          (int)K, w_kmajor ? 1 : 0, (int)epi_in, out.data_ptr(), N, bp,
                          out2.defined() ? out2.data_ptr() : nullptr, N, pp, ldp, cur_stream()),
               "gemm");
  return {out, out2};
}

// da = (dy . w) * GELU'(pre + bias) (w (K, N) k-major: the MLP output projection's weight
// (C, F) read as the input gradient's operand) and db = colsum(da), the fused backward of
// gelu(pre + bias) -> linear: csrc/gemm16.hip's EPI_GELU_BWD epilogue with per-64-row
// column-sum partials.  db goes into db_out (an fp32/bf16 gradient-arena slice) when given.
std::tuple<Tensor, Tensor> gemm_gelu_bwd(const Tensor& dy, const Tensor& w, const Tensor& pre,
                                         const c10::optional<Tensor>& bias,
                                         const c10::optional<Tensor>& db_out, bool pre_is_deriv) {
  check_bf16(dy, "dy");
  check_bf16(w, "w");
  check_bf16(pre, "pre");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "gemm_gelu_bwd: w must be a contiguous (K, N)");
  const int64_t K = w.size(0), N = w.size(1);
  TORCH_CHECK(dy.size(-1) == K, "gemm_gelu_bwd: dy (..., K)");
  auto x2 = dy.reshape({-1, K});
  TORCH_CHECK(x2.stride(1) == 1, "gemm_gelu_bwd: dy must flatten to rows");
  const int64_t M = x2.size(0);
  TORCH_CHECK(M < (1LL << 31) && N < (1 << 30), "gemm_gelu_bwd: shape too large");
  auto pc = pre.reshape({-1, N});
  TORCH_CHECK(pc.size(0) == M && pc.stride(1) == 1, "gemm_gelu_bwd: pre must be (M, N)");
  c10::hip::HIPGuardMasqueradingAsCUDA g(dy.device());
  Tensor bc;
  const void* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_bf16(*bias, "bias");
    bc = bias->contiguous();
    TORCH_CHECK(bc.numel() == N, "gemm_gelu_bwd: bias must have N elements");
    bp = bc.data_ptr();
  }
  auto sizes = pre.sizes().vec();
  auto out = at::empty({M, N}, dy.options());
  const bool given = has_out(db_out, N, "db_out");
  auto db = given ? *db_out : at::empty({N}, bias.has_value() && bias->defined() ? bias->options() : dy.options());
  auto part = at::empty({(long)orion_gemm_colsum_scratch((int)M, (int)N)}, dy.options().dtype(at::kFloat));
  check_launch(orion_gemm(x2.data_ptr(), x2.stride(0), w.data_ptr(), w.stride(0), (int)M, (int)N,
                          (int)K, 1, 3 | (pre_is_deriv ? 0x100 : 0), out.data_ptr(), N, bp, nullptr, 0,
                          pc.data_ptr(), pc.stride(0), cur_stream(), db.data_ptr(), is_f32(db) ? 1 : 0,
                          part.data_ptr<float>()),
               "gemm_gelu_bwd");
  return {out.view(sizes), given ? Tensor() : db};
}

// dgate_up = SwiGLU'(gate_up) applied to dy . w: the fused backward of silu(gate) * up ->
// linear (Llama's down_proj), one in-tree GEMM (K = model dim, N = ffn dim) whose epilogue
// reads the packed (M, 2F) [gate | up] forward projection and writes the packed (M, 2F)
// gradient: the (M, F) input gradient of the SwiGLU is never written and re-read.
Tensor gemm_swiglu_bwd(const Tensor& dy, const Tensor& w, const Tensor& gate_up) {
  check_bf16(dy, "dy");
  check_bf16(w, "w");
  check_bf16(gate_up, "gate_up");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "gemm_swiglu_bwd: w must be a contiguous (K, F)");
  const int64_t K = w.size(0), F = w.size(1);
  TORCH_CHECK(dy.size(-1) == K, "gemm_swiglu_bwd: dy (..., K)");
  auto x2 = dy.reshape({-1, K});
  TORCH_CHECK(x2.stride(1) == 1, "gemm_swiglu_bwd: dy must flatten to rows");
  const int64_t M = x2.size(0);
  auto gu = gate_up.reshape({-1, 2 * F});
  TORCH_CHECK(gu.size(0) == M && gu.stride(1) == 1, "gemm_swiglu_bwd: gate_up must be (M, 2F)");
  TORCH_CHECK(M < (1LL << 31) && F < (1 << 29), "gemm_swiglu_bwd: shape too large");
  c10::hip::HIPGuardMasqueradingAsCUDA g(dy.device());
  auto out = at::empty({M, 2 * F}, dy.options());
  char* o = static_cast<char*>(out.data_ptr());
  check_launch(orion_gemm(x2.data_ptr(), x2.stride(0), w.data_ptr(), w.stride(0), (int)M, (int)F, (int)K, 1,
                          5, o, 2 * F, nullptr, o + F * 2, 2 * F, gu.data_ptr(), gu.stride(0), cur_stream()),
               "gemm_swiglu_bwd");
  auto sizes = gate_up.sizes().vec();
  return out.view(sizes);
}

// ------------------------------------------------------------------ optimizer
void grad_sumsq(const Tensor& g, Tensor out) {
  check_grad_out(g, "grads");
  c10::hip::HIPGuardMasqueradingAsCUDA gd(g.device());
  auto part = at::empty({orion_sumsq_partials()}, g.options().dtype(at::kFloat));
  check_launch(orion_grad_sumsq(g.data_ptr(), g.numel(), is_f32(g), part.data_ptr<float>(),
                                out.data_ptr<float>(), cur_stream()),
               "grad_sumsq");
}

void adamw_flat(Tensor p16, Tensor master, Tensor m, Tensor v, const Tensor& grad,
                const Tensor& decay, const Tensor& hyper, const Tensor& sumsq) {
  check_bf16(p16, "params");
  check_grad_out(grad, "grads");
  TORCH_CHECK(master.scalar_type() == at::kFloat && m.scalar_type() == at::kFloat &&
                  v.scalar_type() == at::kFloat, "optimizer state must be fp32");
  TORCH_CHECK(decay.scalar_type() == at::kByte, "decay flags must be uint8");
  const long n = p16.numel();
  TORCH_CHECK(master.numel() == n && m.numel() == n && v.numel() == n && grad.numel() == n,
              "arena size mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA g(p16.device());
  check_launch(orion_adamw_flat(p16.data_ptr(), master.data_ptr<float>(), m.data_ptr<float>(),
                                v.data_ptr<float>(), grad.data_ptr(), is_f32(grad),
                                decay.data_ptr<uint8_t>(),
                                hyper.data_ptr<float>(), sumsq.data_ptr<float>(), n, cur_stream()),
               "adamw_flat");
}

// ------------------------------------------------------------------ rmsnorm / rope
std::tuple<Tensor, Tensor> rmsnorm_fwd(const Tensor& x, const Tensor& w, double eps) {
  check_bf16(x, "x");
  check_bf16(w, "weight");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto xc = x.contiguous();
  const int C = x.size(-1);
  const int rows = x.numel() / C;
  auto y = at::empty_like(xc);
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  check_launch(orion_rmsnorm_fwd(xc.data_ptr(), w.contiguous().data_ptr(), y.data_ptr(),
                                 rstd.data_ptr<float>(), rows, C, (float)eps, nullptr, nullptr,
                                 cur_stream()),
               "rmsnorm_fwd");
  return {y, rstd};
}

// s = x + r ; y = RMSNorm(s) -> (s, y, rstd)
std::tuple<Tensor, Tensor, Tensor> add_rmsnorm_fwd(const Tensor& x, const Tensor& r, const Tensor& w,
                                                   double eps) {
  check_bf16(x, "x");
  check_bf16(r, "residual");
  check_bf16(w, "weight");
  TORCH_CHECK(x.sizes() == r.sizes(), "add_rmsnorm: shape mismatch");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto xc = x.contiguous(), rc = r.contiguous();
  const int C = x.size(-1);
  const int rows = x.numel() / C;
  auto y = at::empty_like(xc), sum = at::empty_like(xc);
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  check_launch(orion_rmsnorm_fwd(xc.data_ptr(), w.contiguous().data_ptr(), y.data_ptr(),
                                 rstd.data_ptr<float>(), rows, C, (float)eps, rc.data_ptr(),
                                 sum.data_ptr(), cur_stream()),
               "add_rmsnorm_fwd");
  return {sum, y, rstd};
}

// dw_out: the weight's slice of the gradient arena (fp32 or bf16, C elements, written in
// place: ops/grad_sink.py) -- returned as dw; else a fresh tensor of w's dtype.
std::tuple<Tensor, Tensor> rmsnorm_bwd(const Tensor& dy, const Tensor& x, const Tensor& w,
                                       const Tensor& rstd, const c10::optional<Tensor>& dres,
                                       const c10::optional<Tensor>& dw_out) {
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto dyc = dy.contiguous(), xc = x.contiguous();
  const int C = x.size(-1);
  const int rows = x.numel() / C;
  auto dx = at::empty_like(xc);
  Tensor dw;
  if (dw_out.has_value() && dw_out->defined()) {
    check_grad_out(*dw_out, "dw_out");
    TORCH_CHECK(dw_out->is_contiguous() && dw_out->numel() == C, "rmsnorm_bwd: dw_out must be C contiguous elements");
    dw = *dw_out;
  } else {
    dw = at::empty({C}, w.options());
  }
  auto part = at::empty({((long)orion_rmsnorm_bwd_blocks(rows) + 32) * C}, x.options().dtype(at::kFloat));
  Tensor drc;
  if (dres.has_value() && dres->defined()) {
    check_bf16(*dres, "dres");
    drc = dres->contiguous();
  }
  check_launch(orion_rmsnorm_bwd(dyc.data_ptr(), xc.data_ptr(), w.contiguous().data_ptr(),
                                 rstd.data_ptr<float>(), dx.data_ptr(), dw.data_ptr(),
                                 part.data_ptr<float>(), rows, C,
                                 drc.defined() ? drc.data_ptr() : nullptr, is_f32(dw) ? 1 : 0, cur_stream()),
               "rmsnorm_bwd");
  return {dx, dw};
}

// x: (B, T, H, D) view with unit stride on D; returns a contiguous rotated copy.
Tensor rope(const Tensor& x, const Tensor& cosv, const Tensor& sinv, int64_t pos0, double sign) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.stride(3) == 1, "rope: x must be (B, T, H, D) with unit stride on D");
  TORCH_CHECK(cosv.scalar_type() == at::kFloat && cosv.is_contiguous() && sinv.is_contiguous(),
              "rope tables must be contiguous fp32");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  const int B = x.size(0), T = x.size(1), H = x.size(2), D = x.size(3);
  TORCH_CHECK(cosv.size(0) >= T + pos0 && cosv.size(1) == D / 2, "rope table too small");
  auto y = at::empty({B, T, H, D}, x.options());
  check_launch(orion_rope(x.data_ptr(), x.stride(0), x.stride(1), x.stride(2), y.data_ptr(),
                          y.stride(0), y.stride(1), y.stride(2), cosv.data_ptr<float>(),
                          sinv.data_ptr<float>(), B, T, H, D, (int)pos0, (float)sign, cur_stream()),
               "rope");
  return y;
}

// in-place rotation of a strided (B, T, H, D) view (the q|k slice of a packed gradient)
void rope_(Tensor x, const Tensor& cosv, const Tensor& sinv, int64_t pos0, double sign) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.stride(3) == 1, "rope_: x must be (B, T, H, D) with unit stride on D");
  TORCH_CHECK(cosv.scalar_type() == at::kFloat && cosv.is_contiguous() && sinv.is_contiguous(),
              "rope tables must be contiguous fp32");
  c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  const int B = x.size(0), T = x.size(1), H = x.size(2), D = x.size(3);
  TORCH_CHECK(cosv.size(0) >= T + pos0 && cosv.size(1) == D / 2, "rope table too small");
  check_launch(orion_rope(x.data_ptr(), x.stride(0), x.stride(1), x.stride(2), x.data_ptr(),
                          x.stride(0), x.stride(1), x.stride(2), cosv.data_ptr<float>(),
                          sinv.data_ptr<float>(), B, T, H, D, (int)pos0, (float)sign, cur_stream()),
               "rope_");
}

// ------------------------------------------------------------------ attention
void fill_qkv(orion::AttnParams& p, const Tensor& q, const Tensor& k, const Tensor& v) {
  p.q = (const unsigned short*)q.data_ptr();
  p.k = (const unsigned short*)k.data_ptr();
  p.v = (const unsigned short*)v.data_ptr();
  p.q_sb = q.stride(0); p.q_st = q.stride(1); p.q_sh = q.stride(2);
  p.k_sb = k.stride(0); p.k_st = k.stride(1); p.k_sh = k.stride(2);
  p.v_sb = v.stride(0); p.v_st = v.stride(1); p.v_sh = v.stride(2);
  p.B = q.size(0); p.T = q.size(1); p.Hq = q.size(2);
  p.Tk = k.size(1); p.Hkv = k.size(2);
}

void check_attn_inputs(const Tensor& q, const Tensor& k, const Tensor& v) {
  check_bf16(q, "q"); check_bf16(k, "k"); check_bf16(v, "v");
  TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "attention inputs must be (B, T, H, D)");
  TORCH_CHECK(q.stride(3) == 1 && k.stride(3) == 1 && v.stride(3) == 1, "head dim must be contiguous");
  const int D = q.size(3);
  TORCH_CHECK(D == 64 || D == 128, "head dim must be 64 or 128, got ", D);
  TORCH_CHECK(k.size(3) == D && v.size(3) == D && k.sizes() == v.sizes(), "k/v shape mismatch");
  TORCH_CHECK(q.size(2) % k.size(2) == 0, "Hq must be a multiple of Hkv");
  TORCH_CHECK(q.size(0) == k.size(0), "batch mismatch");
  for (const Tensor* t : {&q, &k, &v})
    TORCH_CHECK((t->stride(0) % 8 == 0) && (t->stride(1) % 8 == 0) && (t->stride(2) % 8 == 0) &&
                    ((uintptr_t)t->data_ptr() % 16 == 0),
                "attention inputs need 16-byte aligned rows");
}

std::tuple<Tensor, Tensor> attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, bool causal,
                                    double scale) {
  check_attn_inputs(q, k, v);
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  orion::AttnParams p{};
  fill_qkv(p, q, k, v);
  const int D = q.size(3);
  if (causal) TORCH_CHECK(p.Tk >= p.T, "causal attention needs Tk >= T");
  auto o = at::empty({p.B, p.T, p.Hq, D}, q.options());
  auto lse = at::empty({p.B, p.Hq, p.T}, q.options().dtype(at::kFloat));
  p.o = (unsigned short*)o.data_ptr();
  p.o_sb = o.stride(0); p.o_st = o.stride(1); p.o_sh = o.stride(2);
  p.lse = lse.data_ptr<float>();
  p.scale = (float)scale;
  p.scale_log2 = (float)(scale * 1.4426950408889634);
  check_launch(orion_attn_fwd(p, D, causal, cur_stream()), "attn_fwd");
  return {o, lse};
}

// Backward form: "split" (csrc/attn_bwd_split.hip: dK/dV and dQ kernels, no atomics,
// deterministic) always, except for operands whose 32-bit buffer offsets overflow (one batch's
// Q / dO or one KV head's K / V beyond 2 GB): those take the 64-bit-addressed fused kernel of
// csrc/attention.hip (one pass, fp32-atomic dQ; split measured faster wherever both run:
// 0.632 vs 0.722 ms at B64 T1024 H12 D64, 3.39 vs 4.46 ms at B4 T4096 H32/8 D128).  flags bit 2
// (deterministic) forces split; bit 3 forces the large-operand fallback (its test only).
// column sums of the packed bf16 dQKV starting at dq ([rows][ld], contiguous)
void attn_bias_colsum_packed(const Tensor& dq, const Tensor& out, long rows, long ld) {
  auto part = at::empty({(long)orion_colsum_scratch((int)rows, (int)ld)}, dq.options().dtype(at::kFloat));
  check_launch(orion_colsum_bf16(dq.data_ptr(), out.data_ptr(), part.data_ptr<float>(), (int)rows, (int)ld,
                                 is_f32(out), cur_stream()),
               "attn_bias_colsum");
}

bool attn_bwd_use_split(int D, int64_t flags) {
  if (flags & 4) return true;
  return !(flags & 8);  // bit 3: the large-operand fallback's test
}

// dq/dk/dv: preallocated outputs (may be strided views of one packed buffer)
// bias_grad (optional): the QKV projection's bias gradient, colsum over tokens of the packed
// (B, T, Hq + 2 Hkv, D) dQKV that dq / dk / dv must then be views of.  The split form (MHA,
// D = 64, T % 32 == 0) produces fp32 column sums per 32-token block (AttnParams::bias_part:
// dQ's in the dQ kernel, dK's = 0 and dV's = colsum(dO) in the delta pass) and a two-stage
// fold writes bias_grad (fp32 arena slice or bf16); other shapes and forms sum the packed
// bf16 dQKV.
void attn_bwd(const Tensor& dout, const Tensor& q, const Tensor& k, const Tensor& v,
              const Tensor& o, const Tensor& lse, bool causal, double scale, Tensor dq, Tensor dk,
              Tensor dv, int64_t flags, const c10::optional<Tensor>& bias_grad,
              const c10::optional<Tensor>& rope_cos, const c10::optional<Tensor>& rope_sin,
              int64_t rope_pos0) {
  check_attn_inputs(q, k, v);
  check_bf16(dout, "dout");
  TORCH_CHECK(dout.stride(3) == 1 && o.stride(3) == 1, "dout/o head dim must be contiguous");
  c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  orion::AttnParams p{};
  fill_qkv(p, q, k, v);
  const int D = q.size(3);
  p.o = (unsigned short*)o.data_ptr();
  p.o_sb = o.stride(0); p.o_st = o.stride(1); p.o_sh = o.stride(2);
  p.lse = const_cast<float*>(lse.data_ptr<float>());
  p.scale = (float)scale;
  p.scale_log2 = (float)(scale * 1.4426950408889634);
  p.dout = (const unsigned short*)dout.data_ptr();
  p.do_sb = dout.stride(0); p.do_st = dout.stride(1); p.do_sh = dout.stride(2);
  auto fopts = q.options().dtype(at::kFloat);
  auto delta = at::empty({p.B, p.Hq, p.T}, fopts);
  p.dk = (unsigned short*)dk.data_ptr();
  p.dk_sb = dk.stride(0); p.dk_st = dk.stride(1); p.dk_sh = dk.stride(2);
  p.dv = (unsigned short*)dv.data_ptr();
  p.dv_sb = dv.stride(0); p.dv_st = dv.stride(1); p.dv_sh = dv.stride(2);
  p.flags = (int)flags;
  // rope_cos / rope_sin: dq and dk come out w.r.t. the UNROTATED q / k (the inverse rotation at
  // the split kernels' stores; the other forms run the rope kernel on them afterwards)
  const bool want_rope = rope_cos.has_value() && rope_cos->defined();
  if (want_rope) {
    TORCH_CHECK(rope_sin.has_value() && rope_sin->defined(), "rope_sin missing");
    for (const Tensor* t : {&*rope_cos, &*rope_sin})
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->dim() == 2 &&
                      t->size(1) == D / 2 && t->size(0) >= rope_pos0 + std::max(p.T, p.Tk) && rope_pos0 >= 0,
                  "rope tables must be contiguous fp32 [>= pos0 + T][D / 2]");
    TORCH_CHECK(!has_out(bias_grad, (long)(p.Hq + 2 * p.Hkv) * D, "bias_grad"),
                "rope and the fused QKV bias gradient are exclusive");
    p.rope_cos = rope_cos->data_ptr<float>();
    p.rope_sin = rope_sin->data_ptr<float>();
    p.rope_pos0 = (int)rope_pos0;
  }
  const float* rcos = p.rope_cos;  // kept: p's copies are cleared for the forms below
  const float* rsin = p.rope_sin;
  auto unrope = [&]() {  // the forms without the fused inverse rotation
    if (!want_rope) return;
    for (Tensor* g : {&dq, &dk})
      check_launch(orion_rope(g->data_ptr(), g->stride(0), g->stride(1), g->stride(2), g->data_ptr(),
                              g->stride(0), g->stride(1), g->stride(2), rcos, rsin,
                              (int)g->size(0), (int)g->size(1), (int)g->size(2), D, (int)rope_pos0, -1.f,
                              cur_stream()),
                   "rope (inverse)");
  };
  const long ld = (long)(p.Hq + 2 * p.Hkv) * D;
  const bool want_bias = has_out(bias_grad, ld, "bias_grad");
  Tensor bpart;
  if (want_bias) {
    const long e = dq.element_size();
    TORCH_CHECK(p.T == p.Tk && dq.stride(1) == ld && dk.stride(1) == ld && dv.stride(1) == ld &&
                    dq.stride(0) == p.T * ld && dq.stride(2) == D && dk.stride(2) == D &&
                    dv.stride(2) == D &&
                    (char*)dk.data_ptr() == (char*)dq.data_ptr() + p.Hq * D * e &&
                    (char*)dv.data_ptr() == (char*)dk.data_ptr() + p.Hkv * D * e,
                "bias_grad needs dq / dk / dv to be views of one packed (B, T, Hq + 2 Hkv, D) dQKV");
  }
  if (attn_bwd_use_split(D, flags)) {
    p.dq = (unsigned short*)dq.data_ptr();
    p.dq_sb = dq.stride(0); p.dq_st = dq.stride(1); p.dq_sh = dq.stride(2);
    const long prow = (long)p.B * ((p.T + 31) / 32);
    if (want_bias && D == 64) {
      bpart = at::empty({prow * ld + 16 * ld}, fopts);  // partials + the fold's scratch
      p.bias_part = bpart.data_ptr<float>();
      p.bias_ld = (int)ld;
    }
    int rc = orion_attn_bwd_split(p, D, causal, delta.data_ptr<float>(), cur_stream());
    if (rc == -3) {  // no in-kernel column sums for this form: plain kernels, summed below
      p.bias_part = nullptr;
      rc = orion_attn_bwd_split(p, D, causal, delta.data_ptr<float>(), cur_stream());
    }
    if (rc != -2) {  // -2: operands beyond the split kernels' 32-bit offsets -> fused form
      check_launch(rc, "attn_bwd_split");
      if (want_bias) {
        if (p.bias_part)
          check_launch(orion_colsum_partials2(p.bias_part, p.bias_part + prow * ld, bias_grad->data_ptr(),
                                              (int)prow, (int)ld, is_f32(*bias_grad), cur_stream()),
                       "attn_bias_colsum");
        else
          attn_bias_colsum_packed(dq, *bias_grad, p.B * p.T, ld);
      }
      return;
    }
    p.bias_part = nullptr;
  }
  p.rope_cos = p.rope_sin = nullptr;
  auto dq_acc = at::empty({p.B, p.Hq, p.T, D}, fopts);
  p.dq_acc = dq_acc.data_ptr<float>();
  check_launch(orion_attn_bwd(p, D, causal, delta.data_ptr<float>(), cur_stream()), "attn_bwd");
  check_launch(orion_attn_dq_convert(dq_acc.data_ptr<float>(), dq.data_ptr(), dq.stride(0),
                                     dq.stride(1), dq.stride(2), p.B, p.Hq, p.T, D, cur_stream()),
               "attn_dq_convert");
  if (want_bias) attn_bias_colsum_packed(dq, *bias_grad, p.B * p.T, ld);
  unrope();
}

}  // namespace

TORCH_LIBRARY(orion_amd, m) {
  m.def("layernorm_fwd(Tensor x, Tensor w, Tensor? b, float eps) -> (Tensor, Tensor, Tensor)");
  m.def("layernorm_bwd(Tensor dy, Tensor x, Tensor w, Tensor mean, Tensor rstd, bool has_bias, Tensor? dres=None, bool want_dx_colsum=False, Tensor(a!)? dw_out=None, Tensor(b!)? db_out=None, Tensor(c!)? dxs_out=None) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("embed_layernorm_fwd(Tensor idx, Tensor wte, Tensor wpe, Tensor w, Tensor? b, float eps) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("embed_scatter_add_(Tensor dx, Tensor idx, Tensor(a!) out) -> ()");
  m.def("embed_id_error(int device) -> int", &embed_id_error);
  m.def("batch_sum_(Tensor x, Tensor(a!) out) -> ()");
  m.def("add_layernorm_fwd(Tensor x, Tensor r, Tensor w, Tensor? b, float eps, Tensor? rbias=None) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("bias_gelu_fwd(Tensor x, Tensor? b) -> Tensor");
  m.def("bias_gelu_bwd(Tensor dy, Tensor x, Tensor? b, Tensor(a!)? db_out=None) -> (Tensor, Tensor)");
  m.def("colsum(Tensor m, Tensor(a!)? out=None) -> Tensor");
  m.def("swiglu_fwd(Tensor gu) -> Tensor");
  m.def("swiglu_bwd(Tensor dy, Tensor gu) -> Tensor");
  m.def("scale_(Tensor(a!) x, Tensor s) -> ()");
  m.def("slab_sum(Tensor slabs, Tensor? scale=None) -> Tensor");
  m.def("wgrad(Tensor dy, Tensor x, Tensor? scale=None, int splits=0) -> Tensor");
  m.def("wgrad_into(Tensor dy, Tensor x, Tensor? scale, Tensor(a!) out, bool accumulate, int splits=0) -> ()");
  m.def("wgrad_splits(int M, int N1, int N2) -> int", &wgrad_splits);  // host-only helper
  m.def("wgrad_tail_rows(int M, int N1, int N2) -> (int, int)", &wgrad_tail_rows);  // host-only
  m.def("gemm_diag(int flags) -> int", &gemm_diag);                   // host-only helper
  m.def("xent_fwd_bwd(Tensor(a!) logits, Tensor targets, int ignore_index) -> Tensor");
  m.def("lmhead_fwd(Tensor x, Tensor w, Tensor targets, int ignore_index, Tensor(a!) cref) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("lmhead_bwd_prep(Tensor x, Tensor targets, int ignore_index, int V, Tensor invz, Tensor inv_n, Tensor g, bool transposed=False) -> (Tensor, Tensor)");
  m.def("gemm_rowscale(Tensor e, Tensor w, Tensor srow) -> Tensor");
  m.def("gemm_rope(Tensor x, Tensor w, Tensor cos, Tensor sin, int pos0, int T, int rope_cols, int D) -> Tensor");
  m.def("gemm_swiglu(Tensor x, Tensor w) -> Tensor[]");
  m.def("linear_residual(Tensor x, Tensor w, Tensor? bias, Tensor? r) -> Tensor");
  m.def("gemm(Tensor x, Tensor w, bool w_kmajor, int epi, Tensor? bias=None, Tensor? pre=None) -> (Tensor, Tensor)");
  m.def("gemm_gelu_bwd(Tensor dy, Tensor w, Tensor pre, Tensor? bias=None, Tensor(a!)? db_out=None, bool pre_is_deriv=False) -> (Tensor, Tensor)");
  m.def("gemm_swiglu_bwd(Tensor dy, Tensor w, Tensor gate_up) -> Tensor");
  m.def("grad_sumsq(Tensor g, Tensor(a!) out) -> ()");
  m.def("adamw_flat(Tensor(a!) p16, Tensor(b!) master, Tensor(c!) m, Tensor(d!) v, Tensor g, Tensor decay, Tensor hyper, Tensor sumsq) -> ()");
  m.def("rmsnorm_fwd(Tensor x, Tensor w, float eps) -> (Tensor, Tensor)");
  m.def("rmsnorm_bwd(Tensor dy, Tensor x, Tensor w, Tensor rstd, Tensor? dres=None, Tensor(a!)? dw_out=None) -> (Tensor, Tensor)");
  m.def("add_rmsnorm_fwd(Tensor x, Tensor r, Tensor w, float eps) -> (Tensor, Tensor, Tensor)");
  m.def("rope(Tensor x, Tensor cos, Tensor sin, int pos0, float sign) -> Tensor");
  m.def("rope_(Tensor(a!) x, Tensor cos, Tensor sin, int pos0, float sign) -> ()");
  m.def("attn_fwd(Tensor q, Tensor k, Tensor v, bool causal, float scale) -> (Tensor, Tensor)");
  m.def("attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, bool causal, float scale, Tensor(a!) dq, Tensor(b!) dk, Tensor(c!) dv, int flags=0, Tensor(d!)? bias_grad=None, Tensor? rope_cos=None, Tensor? rope_sin=None, int rope_pos0=0) -> ()");
}

TORCH_LIBRARY_IMPL(orion_amd, CUDA, m) {
  m.impl("layernorm_fwd", &layernorm_fwd);
  m.impl("layernorm_bwd", &layernorm_bwd);
  m.impl("add_layernorm_fwd", &add_layernorm_fwd);
  m.impl("embed_layernorm_fwd", &embed_layernorm_fwd);
  m.impl("embed_scatter_add_", &embed_scatter_add_);
  m.impl("batch_sum_", &batch_sum_);
  m.impl("bias_gelu_fwd", &bias_gelu_fwd);
  m.impl("bias_gelu_bwd", &bias_gelu_bwd);
  m.impl("colsum", &colsum);
  m.impl("swiglu_fwd", &swiglu_fwd);
  m.impl("swiglu_bwd", &swiglu_bwd);
  m.impl("scale_", &scale_);
  m.impl("slab_sum", &slab_sum);
  m.impl("wgrad", &wgrad);
  m.impl("wgrad_into", &wgrad_into);
  m.impl("xent_fwd_bwd", &xent_fwd_bwd);
  m.impl("lmhead_fwd", &lmhead_fwd);
  m.impl("lmhead_bwd_prep", &lmhead_bwd_prep);
  m.impl("gemm_rowscale", &gemm_rowscale);
  m.impl("gemm_rope", &gemm_rope);
  m.impl("gemm_swiglu", &gemm_swiglu);
  m.impl("linear_residual", &linear_residual);
  m.impl("gemm", &gemm);
  m.impl("gemm_gelu_bwd", &gemm_gelu_bwd);
  m.impl("gemm_swiglu_bwd", &gemm_swiglu_bwd);
  m.impl("grad_sumsq", &grad_sumsq);
  m.impl("adamw_flat", &adamw_flat);
  m.impl("rmsnorm_fwd", &rmsnorm_fwd);
  m.impl("rmsnorm_bwd", &rmsnorm_bwd);
  m.impl("add_rmsnorm_fwd", &add_rmsnorm_fwd);
  m.impl("rope", &rope);
  m.impl("rope_", &rope_);
  m.impl("attn_fwd", &attn_fwd);
  m.impl("attn_bwd", &attn_bwd);
}
