"""KV-cached generation (llmtrain.inference) against the reference's notebook sampler
(notebooks/trained_vs_random_completion.ipynb ``generate_text``: full-context recompute per
token, crop to block_size, temperature / top-k / multinomial), plus the ``generate`` CLI."""

from __future__ import annotations

import json
from pathlib import Path

import pytest
import torch

from llmtrain.cli import main
from llmtrain.inference import KVCache, forward_cached, generate, sample_next_token
from llmtrain.models.gpt import GPT


def _model(block: int = 16) -> GPT:
    torch.manual_seed(0)
    m = GPT(vocab_size=64, block_size=block, d_model=32, n_layers=2, n_heads=4, d_ff=64, dropout=0.0)
    return m.double().eval()


def _notebook_loop(model: GPT, x: torch.Tensor, n: int, temperature: float, top_k: int | None) -> torch.Tensor:
    """The notebook's generate_text body, verbatim in behaviour."""
    for _ in range(n):
        x_cond = x[:, -model.block_size :]
        with torch.no_grad():
            next_logits = model(x_cond)[:, -1, :]
        if temperature <= 0:
            nxt = torch.argmax(next_logits, dim=-1, keepdim=True)
        else:
            next_logits = next_logits / temperature
            if top_k is not None and top_k > 0:
                values, _ = torch.topk(next_logits, k=min(top_k, next_logits.size(-1)))
                cutoff = values[:, -1].unsqueeze(-1)
                next_logits = torch.where(next_logits < cutoff, torch.full_like(next_logits, float("-inf")), next_logits)
            nxt = torch.multinomial(torch.softmax(next_logits, dim=-1), num_samples=1)
        x = torch.cat((x, nxt), dim=1)
    return x


def test_cached_forward_matches_full_forward() -> None:
    model = _model()
    ids = torch.randint(0, 64, (2, 10))
    cache = KVCache.allocate(model, 2, dtype=torch.float64, device=torch.device("cpu"))
    logits = forward_cached(model, ids[:, :6], cache)
    torch.testing.assert_close(logits, model(ids[:, :6])[:, -1], rtol=1e-10, atol=1e-10)
    for t in range(6, 10):  # one token at a time, then a 2-token chunk is covered by the prefill
        logits = forward_cached(model, ids[:, t : t + 1], cache)
        torch.testing.assert_close(logits, model(ids[:, : t + 1])[:, -1], rtol=1e-10, atol=1e-10)
    assert cache.length == 10


@pytest.mark.parametrize("temperature,top_k", [(0.0, None), (0.8, 40), (1.3, 5), (0.7, None)])
def test_generate_matches_notebook_sampler_past_block_size(temperature: float, top_k: int | None) -> None:
    model = _model(block=16)
    prompt = torch.randint(0, 64, (1, 5))
    torch.manual_seed(7)
    want = _notebook_loop(model, prompt, 20, temperature, top_k)  # 25 tokens > block_size 16
    torch.manual_seed(7)
    got = generate(model, prompt, 20, temperature=temperature, top_k=top_k)
    assert torch.equal(got, want)
    torch.manual_seed(7)
    assert torch.equal(generate(model, prompt, 20, temperature=temperature, top_k=top_k, use_cache=False), want)


def test_top_k_one_is_greedy_and_eos_stops() -> None:
    logits = torch.randn(3, 50, dtype=torch.float64)
    assert torch.equal(sample_next_token(logits, temperature=1.0, top_k=1), logits.argmax(-1, keepdim=True))
    model = _model()
    prompt = torch.randint(0, 64, (2, 4))
    greedy = generate(model, prompt, 6, temperature=0.0)
    eos = int(greedy[0, 4])  # the first generated token of row 0
    out = generate(model, prompt, 6, temperature=0.0, eos_token_id=eos)
    assert out[0, 4] == eos and (out[0, 4:] == eos).all()


def test_generate_cli_from_trained_checkpoint(in_tmp: Path) -> None:
    cfg = {
        "schema_version": 1,
        "run": {"name": "gen", "seed": 3, "device": "cpu"},
        "model": {"name": "gpt", "vocab_size": 256, "block_size": 16, "d_model": 64, "n_layers": 1, "n_heads": 2,
                  "d_ff": 128, "dropout": 0.0},
        "data": {"name": "synthetic_tokens", "num_workers": 0, "extra": {"train_sequences": 32, "val_sequences": 4}},
        "trainer": {"max_steps": 2, "warmup_steps": 0, "micro_batch_size": 4, "grad_accum_steps": 1,
                    "log_every_steps": 1, "eval_every_steps": 2, "save_every_steps": 2},
        "ddp": {"enabled": False}, "mlflow": {"enabled": False},
        "logging": {"log_to_file": False}, "output": {"root_dir": "runs", "run_id": "genrun"},
    }
    import yaml

    Path("cfg.yaml").write_text(yaml.safe_dump(cfg))
    assert main(["train", "--config", "cfg.yaml", "--json"]) == 0
    argv = ["generate", "--config", "cfg.yaml", "--checkpoint", "genrun", "--prompt", "hello", "--prompt", "ab",
            "--max-new-tokens", "5", "--top-next", "3", "--json"]
    import contextlib
    import io

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        assert main(argv) == 0
    out = json.loads(buf.getvalue())
    assert out["checkpoint"].endswith("step_000002.pt")
    assert [r["prompt"] for r in out["results"]] == ["hello", "ab"]
    assert all(r["completion"].startswith(r["prompt"]) for r in out["results"])
    assert len(out["results"][0]["top_next"]) == 3
    # an unknown checkpoint is a runtime failure (exit 1), a non-causal model a usage error (exit 2)
    assert main(["generate", "--config", "cfg.yaml", "--checkpoint", "nope", "--prompt", "x"]) == 1


@pytest.mark.gpu
def test_cached_decode_on_gpu(gpu_device) -> None:  # type: ignore[no-untyped-def]
    torch.manual_seed(0)
    model = GPT(vocab_size=512, block_size=64, d_model=128, n_layers=2, n_heads=2, d_ff=256, dropout=0.0)
    model = model.to(gpu_device).eval()
    ids = torch.randint(0, 512, (3, 40), device=gpu_device)
    cache = KVCache.allocate(model, 3, dtype=torch.float32, device=gpu_device)
    forward_cached(model, ids[:, :30], cache)
    for t in range(30, 40):
        got = forward_cached(model, ids[:, t : t + 1], cache)
        with torch.no_grad():
            want = model(ids[:, : t + 1])[:, -1]
        torch.testing.assert_close(got, want, rtol=1e-3, atol=1e-3)
    out = generate(model, ids[:, :8], 70, temperature=0.9, top_k=20, autocast_dtype=torch.bfloat16)
    assert out.shape == (3, 78) and int(out.max()) < 512


def test_graph_decoder_static_step_matches_full_forward() -> None:
    """The static-shape step the hipGraph records (full-capacity masked attention, device-side
    position) equals the full forward at every position, here run eagerly on CPU."""
    from llmtrain.inference import GraphDecoder

    model = _model(block=16)
    ids = torch.randint(0, 64, (3, 16))
    dec = GraphDecoder(model, 3)
    assert not dec.use_graph
    logits = dec.prefill(ids[:, :5])
    torch.testing.assert_close(logits, model(ids[:, :5])[:, -1], rtol=1e-10, atol=1e-10)
    for t in range(5, 16):
        logits = dec.decode(ids[:, t : t + 1])
        torch.testing.assert_close(logits, model(ids[:, : t + 1])[:, -1], rtol=1e-10, atol=1e-10)
    assert dec.length == 16
    with pytest.raises(ValueError, match="full"):
        dec.decode(ids[:, :1])


@pytest.mark.parametrize("temperature,top_k", [(0.0, None), (0.9, 8)])
def test_generate_graph_path_matches_cached_path(temperature: float, top_k: int | None) -> None:
    model = _model(block=16)
    prompt = torch.randint(0, 64, (2, 4))
    torch.manual_seed(11)
    want = generate(model, prompt, 18, temperature=temperature, top_k=top_k)  # crosses block_size
    torch.manual_seed(11)
    got = generate(model, prompt, 18, temperature=temperature, top_k=top_k, use_graph=True)
    assert torch.equal(got, want)
