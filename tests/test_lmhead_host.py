"""Host-side logic of the LM-head + cross-entropy path (orion_amd/ops/xent.py), CPU only:
which inputs take the exp-epilogue kernels, and the per-weight exp-reference table (one
device scalar per LM-head weight, bounded, fresh in deterministic mode)."""
import torch

from orion_amd.ops import xent as X


def test_exp_path_eligibility_is_gpu_bf16_aligned_only():
    x = torch.zeros(64, 768, dtype=torch.bfloat16)
    w = torch.zeros(1024, 768, dtype=torch.bfloat16)
    assert not X.lmhead_exp_eligible(x, w)            # CPU tensors: the row-pass / reference path
    assert not X.lmhead_exp_eligible(x.float(), w)


def test_exp_reference_table_per_weight_and_bounded(monkeypatch):
    monkeypatch.setattr(X, "_CREF", {})
    dev = torch.device("cpu")
    w1, w2 = torch.zeros(8, 64), torch.zeros(8, 64)
    a, b = X._cref(dev, w1), X._cref(dev, w2)
    assert a is not b and X._cref(dev, w1) is a       # one scalar per weight storage, reused
    a.fill_(3.0)
    assert float(X._cref(dev, w2)) == 0.0             # another model's forwards do not feed it
    keep = [torch.zeros(4) for _ in range(100)]        # live storages: distinct data pointers
    for t in keep:
        X._cref(dev, t)
    assert len(X._CREF) <= 64                          # freed storages are reused: bounded


def test_exp_reference_fresh_in_deterministic_mode(monkeypatch):
    from orion_amd.ops import determinism
    monkeypatch.setattr(X, "_CREF", {})
    monkeypatch.setattr(determinism, "deterministic", lambda: True)
    w = torch.zeros(8, 64)
    a = X._cref(torch.device("cpu"), w)
    a.fill_(5.0)
    assert float(X._cref(torch.device("cpu"), w)) == 0.0
    assert X._CREF == {}
