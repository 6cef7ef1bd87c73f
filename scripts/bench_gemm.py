#!/usr/bin/env python3
"""GEMM microbenchmark on the GPT-2-124M training shapes (M = 64 x 1024 tokens):
csrc/gemm16.hip (with its fused epilogues) vs hipBLASLt through PyTorch (committed TunableOp
table loaded) plus the separate HIP epilogue kernels it needs.  Interleaved rounds in one
process, median per variant; one JSON line per shape.

usage: python scripts/bench_gemm.py [--M 65536] [--iters 20] [--check] [--cfgs p,s]
(cfgs: p gemm16 persistent, s one workgroup per item)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fns, iters):
    """fns: dict name -> callable; interleaved rounds, median ms per name."""
    for f in fns.values():
        for _ in range(3):
            f()
    torch.cuda.synchronize()
    ts = {k: [] for k in fns}
    for _ in range(iters):
        for k, f in fns.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            b.synchronize()
            ts[k].append(a.elapsed_time(b))
    return {k: sorted(v)[len(v) // 2] for k, v in ts.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--check", action="store_true", help="compare outputs against torch")
    ap.add_argument("--cfgs", default="p", help="comma list of in-tree variants to time: p = gemm16's "
                    "persistent walk (default), s = one workgroup per work item (gemm_diag(64))")
    ap.add_argument("--square", type=int, default=0, help="also time an NT GEMM of this cube size")
    ap.add_argument("--only", default="", help="comma list of shape names to run")
    ap.add_argument("--llama", action="store_true", help="Llama-2-7B shapes (M = 16,384 tokens) instead")
    ap.add_argument("--step-data", action="store_true",
                    help="operands distributed like the training step's (activations N(0, 1), weights "
                         "N(0, 0.02^2)) instead of N(0, 0.5^2) for both: the chip's clock depends on the data")
    a = ap.parse_args()
    from orion_amd.ops._ext import C, load_ext
    from orion_amd.tuning import use_tuned_gemms
    load_ext(required=True)
    use_tuned_gemms()
    ops = C()
    M = a.M
    g = torch.Generator(device="cuda").manual_seed(0)
    rnd = lambda *s: (torch.randn(*s, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    # (name, kind, N, K, epi): fwd = x (M,K) . W(N,K)^T; dgrad = dy (M,K) . W(K,N)
    shapes = [("qkv_fwd", "fwd", 2304, 768, 1), ("attnproj_fwd", "fwd", 768, 768, 0),
              ("fc_fwd+bias+gelu", "fwd", 3072, 768, 2), ("mlpproj_fwd", "fwd", 768, 3072, 0),
              ("lmhead_fwd", "fwd", 50304, 768, 0), ("lmhead_exp", "fwd", 50304, 768, 6),
              ("qkv_dgrad", "dgrad", 768, 2304, 0), ("attnproj_dgrad", "dgrad", 768, 768, 0),
              ("fc_dgrad", "dgrad", 768, 3072, 0), ("mlpproj_dgrad+gelu_bwd", "dgrad", 3072, 768, 3),
              # 5: gemm_gelu_bwd (GELU'(pre + b) and the bias gradient in the epilogue) against
              # the unfused dgrad GEMM + bias_gelu_bwd (which also sums the bias gradient)
              ("mlpproj_dgrad+gelu_bwd+db", "dgrad", 3072, 768, 5),
              ("lmhead_dgrad", "dgrad", 768, 50304, 0), ("lmhead_dgrad_rowscale", "dgrad", 768, 50304, 7),
              # the fused shapes without their epilogue arithmetic (price of the epilogue)
              ("fc_fwd_plain", "fwd", 3072, 768, 0), ("fc_fwd+bias", "fwd", 3072, 768, 1),
              ("mlpproj_dgrad_plain", "dgrad", 3072, 768, 0)]
    if a.llama:
        shapes = [("l_qkv_fwd", "fwd", 12288, 4096, 0), ("l_o_fwd", "fwd", 4096, 4096, 0),
                  ("l_gateup_fwd", "fwd", 22016, 4096, 0), ("l_down_fwd", "fwd", 4096, 11008, 0),
                  ("l_lmhead_fwd", "fwd", 32000, 4096, 0),
                  ("l_qkv_dgrad", "dgrad", 4096, 12288, 0), ("l_o_dgrad", "dgrad", 4096, 4096, 0),
                  ("l_gateup_dgrad", "dgrad", 4096, 22016, 0), ("l_down_dgrad", "dgrad", 11008, 4096, 0),
                  ("l_lmhead_dgrad", "dgrad", 4096, 32000, 0)]
    if a.square:
        shapes = [(f"square{a.square}", "fwd", a.square, a.square, 0)] + shapes
    if a.only:
        shapes = [sh for sh in shapes if sh[0] in a.only.split(",")]
    cfgs = a.cfgs.split(",")
    tot = {"hip": 0.0, "blas": 0.0}
    for name, kind, N, K, epi in shapes:
        if name.startswith("square"):
            M = a.square
        else:
            M = a.M
        x = rnd(M, K)
        w = rnd(N, K) if kind == "fwd" else rnd(K, N)
        if a.step_data:
            x = (x.float() * 2.0).bfloat16()
            w = (w.float() * 0.04).bfloat16()
        b = rnd(N) if epi in (1, 2, 5) else None
        pre = rnd(M, N) if epi in (3, 5) else None
        if epi == 6:  # LM head: exp epilogue + fold (csrc/lmhead.hip) vs hipBLASLt logits
            tg = torch.randint(0, N, (M,), device="cuda", generator=g)
            cref = torch.zeros(1, device="cuda")
            hip = lambda: ops.lmhead_fwd(x, w, tg, -1, cref)
            blas = lambda: torch.nn.functional.linear(x, w)
        elif kind == "fwd":
            hip = lambda: ops.gemm(x, w, False, epi, b, None)
            if epi == 2:
                blas = lambda: ops.bias_gelu_fwd(torch.nn.functional.linear(x, w), b)
            else:
                blas = lambda: torch.nn.functional.linear(x, w, b)
        elif epi == 7:  # LM head input gradient with the per-row softmax scale in the epilogue
            srow = torch.rand(M, device="cuda", generator=g)
            hip = lambda: ops.gemm_rowscale(x, w, srow)
            blas = lambda: x @ w
        else:
            hip = lambda: ops.gemm(x, w, True, epi, None, pre)
            if epi == 5:
                hip = lambda: ops.gemm_gelu_bwd(x, w, pre, b, None)
                blas = lambda: ops.bias_gelu_bwd(x @ w, pre, b, None)
            elif epi == 3:
                # the unfused path: dgrad GEMM, then the GELU backward kernel (x = pre, no bias)
                blas = lambda: ops.bias_gelu_bwd(x @ w, pre, None, None)
            else:
                blas = lambda: x @ w
        def with_cfg(c, f):
            def run():
                ops.gemm_diag({"s": 64}.get(c, 0))
                return f()
            return run
        fns = {f"hip{c}": with_cfg(c, hip) for c in cfgs}
        fns["blas"] = blas
        t = timeit(fns, a.iters)
        t["hip"] = t[f"hip{cfgs[0]}"]
        flop = 2.0 * M * N * K
        rec = {"shape": name, "M": M, "N": N, "K": K, "epi": epi,
               "hip_ms": round(t["hip"], 4), "blas_ms": round(t["blas"], 4),
               "hip_TFs": round(flop / t["hip"] / 1e9, 1), "blas_TFs": round(flop / t["blas"] / 1e9, 1)}
        for c in cfgs[1:]:
            rec[f"cfg{c}_TFs"] = round(flop / t[f"hip{c}"] / 1e9, 1)
        if a.check and epi not in (6, 7):
            ref = (x.float() @ (w.float().t() if kind == "fwd" else w.float()))
            if b is not None and epi != 5:
                ref = ref + b.float()
            got = with_cfg(cfgs[0], hip)()
            o = got[0].float()
            if epi in (3, 5):
                from orion_amd.ops import reference as R
                gp = torch.func.grad(lambda z: R.gelu_tanh(z).sum())
                ref = ref * gp(pre.float() + (b.float() if epi == 5 else 0))
                if epi == 5:
                    rec["rel_err_db"] = float((got[1].float() - ref.sum(0)).norm() / ref.sum(0).norm())
            rec["rel_err"] = float((o - ref).norm() / ref.norm())
            if epi == 2:
                from orion_amd.ops import reference as R
                rec["rel_err_gelu"] = float((got[1].float() - R.gelu_tanh(ref)).norm() / R.gelu_tanh(ref).norm())
        tot["hip"] += t["hip"]
        tot["blas"] += t["blas"]
        print(json.dumps(rec), flush=True)
        del x, w, b, pre
    print(json.dumps({"total_hip_ms": round(tot["hip"], 3), "total_blas_ms": round(tot["blas"], 3)}))


if __name__ == "__main__":
    main()
