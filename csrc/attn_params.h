// Parameter block shared by csrc/attention.hip and csrc/bindings.cpp.
#pragma once

namespace orion {

struct AttnParams {
  const unsigned short* q;  // bf16 bits
  const unsigned short* k;
  const unsigned short* v;
  unsigned short* o;
  float* lse;  // [B][Hq][T], base-2 log-sum-exp of scaled scores
  long q_sb, q_st, q_sh;
  long k_sb, k_st, k_sh;
  long v_sb, v_st, v_sh;
  long o_sb, o_st, o_sh;
  int B, T, Tk, Hq, Hkv;
  float scale;       // softmax scale (1/sqrt(D))
  float scale_log2;  // scale * log2(e)
  // backward
  const unsigned short* dout;
  long do_sb, do_st, do_sh;
  const float* delta;  // [B][Hq][T] = rowsum(dO * O) (written by attn_bwd_dq4_kernel at D = 64)
  float* dq_acc;       // [B][Hq][T][D] fp32
  unsigned short* dk;
  long dk_sb, dk_st, dk_sh;
  unsigned short* dv;
  long dv_sb, dv_st, dv_sh;
  unsigned short* dq;  // bf16 dQ (split backward: written directly, no fp32 accumulator)
  long dq_sb, dq_st, dq_sh;
  int flags;  // 1 = skip dQ atomics (diagnostic), 4 = deterministic (split backward), 8 = fused
  // split backward, packed self-attention (T == Tk, MHA, D = 64, T % 32 == 0): column sums of
  // dQ | dK | dV over every 32-token block, [B * T / 32][bias_ld] fp32 (bias_ld = 3 Hq D) -- dQ's
  // from the dQ kernel, dK's (identically 0) and dV's (= those of dO) from the delta pass -- so
  // the QKV projection's bias gradient needs no pass over the packed dQKV
  float* bias_part;
  int bias_ld;
  // split backward: the inverse rotary embedding of dQ / dK at their stores (the attention ran
  // on rope(q), rope(k); the caller wants the gradient w.r.t. the unrotated projection).
  // cos / sin tables [positions][D / 2] fp32, position of token t = t + rope_pos0; null: none.
  const float* rope_cos;
  const float* rope_sin;
  int rope_pos0;
};

}  // namespace orion
