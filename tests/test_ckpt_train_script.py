"""train.py / sample.py / checkpoint round trip on CPU (nanoGPT-compatible surface)."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, cwd, env=None):
    r = subprocess.run([sys.executable] + args, cwd=cwd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_train_resume_sample(tmp_path):
    out = str(tmp_path / "out")
    common = ["--device=cpu", "--model=gpt2-tiny", "--n_layer=2", "--n_head=4", "--n_embd=128",
              "--block_size=32", "--batch_size=2", "--gradient_accumulation_steps=2",
              "--eval_iters=1", f"--out_dir={out}", "--dataset="]
    s = _run([os.path.join(ROOT, "train.py")] + common + ["--max_iters=4", "--eval_interval=2"], str(tmp_path))
    assert "step 4" in s
    ck = torch.load(os.path.join(out, "ckpt.pt"), map_location="cpu", weights_only=True)
    assert set(ck) >= {"model", "optimizer", "model_args", "iter_num", "best_val_loss", "config"}
    assert ck["iter_num"] == 4 and ck["model_type"] == "gpt2"
    assert "lm_head.weight" in ck["model"] and "transformer.wte.weight" in ck["model"]
    s = _run([os.path.join(ROOT, "train.py")] + common + ["--init_from=resume", "--max_iters=6",
                                                         "--eval_interval=3"], str(tmp_path))
    assert "iter 4" in s and "step 6" in s
    s = _run([os.path.join(ROOT, "sample.py"), f"--out_dir={out}", "--device=cpu", "--num_samples=1",
              "--max_new_tokens=4", "--start=ids:1,2"], str(tmp_path))
    assert "[1, 2," in s


def test_nanogpt_py_config_is_parsed_not_executed(tmp_path):
    sys.path.insert(0, ROOT)
    import train
    cfgf = tmp_path / "cfg.py"
    cfgf.write_text("batch_size = 7\nlearning_rate = 1e-3  # comment\nimport os\nos.system('false')\n")
    cfg = train.parse_config([str(cfgf), "--max_iters=3"])
    assert cfg["batch_size"] == 7 and cfg["learning_rate"] == 1e-3 and cfg["max_iters"] == 3


def test_train_reports_to_orion(tmp_path):
    res = tmp_path / "res.json"
    res.write_text("")
    env = dict(os.environ, METAOPT_RESULTS_PATH=str(res))
    _run([os.path.join(ROOT, "train.py"), "--device=cpu", "--model=gpt2-tiny", "--n_layer=1", "--n_head=2",
          "--n_embd=64", "--block_size=16", "--batch_size=2", "--gradient_accumulation_steps=1",
          "--max_iters=2", "--eval_interval=2", "--eval_iters=1", f"--out_dir={tmp_path}/o", "--dataset="],
         str(tmp_path), env=env)
    import json
    (r,) = json.loads(res.read_text())
    assert r["type"] == "objective" and r["name"] == "val_loss" and r["value"] > 0


def test_llama_checkpoint_roundtrip(tmp_path):
    sys.path.insert(0, ROOT)
    from orion_amd.models import build_model
    from orion_amd.train.ckpt import build_model_from_checkpoint, load_checkpoint, save_checkpoint
    from orion_amd.train.engine import Trainer
    torch.manual_seed(0)
    m = build_model("llama-tiny")
    tr = Trainer(m)
    x = torch.randint(0, 512, (2, 16))
    tr.step([(x, x)])
    p = save_checkpoint(str(tmp_path / "ck.pt"), tr, 1.0, {"a": 1})
    m2 = build_model_from_checkpoint(load_checkpoint(p))
    for (n, a), (_, b) in zip(m.named_parameters(), m2.named_parameters()):
        assert torch.allclose(a.float(), b.float()), n


def test_train_profiler_trace(tmp_path):
    """profile_steps > 0 writes a Chrome trace of that many steps (SURVEY.md §5 tracing)."""
    _run([os.path.join(ROOT, "train.py"), "--device=cpu", "--model=gpt2-tiny", "--n_layer=1", "--n_head=2",
          "--n_embd=64", "--block_size=16", "--batch_size=2", "--gradient_accumulation_steps=1",
          "--max_iters=4", "--eval_interval=4", "--eval_iters=1", f"--out_dir={tmp_path}/o", "--dataset=",
          "--profile_start=1", "--profile_steps=2"], str(tmp_path))
    import json
    trace = json.loads((tmp_path / "o" / "trace_rank0.json").read_text())
    assert trace["traceEvents"]
