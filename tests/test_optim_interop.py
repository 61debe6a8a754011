"""Two-way optimizer-state interop between :class:`FusedAdamW` and ``torch.optim.AdamW``.

Reference contract: the checkpoint's ``optimizer_state_dict`` is a ``torch.optim.AdamW`` state
(``/root/reference/src/llmtrain/training/trainer.py:93-97``, ``training/checkpoint.py:53-68``), so a
checkpoint written by the fused optimizer must resume under torch AdamW (module path, reference
trainer) and vice versa — with a per-parameter ``step`` that advances by exactly one per step.
"""

from __future__ import annotations

import copy
import io

import torch
import torch.nn.functional as F

from llmtrain.models.gpt import GPT
from llmtrain.training.optim import FusedAdamW

from conftest import minimal_payload

V = 100


def _models():  # type: ignore[no-untyped-def]
    torch.manual_seed(0)
    plain = GPT(vocab_size=V, block_size=16, d_model=64, n_layers=2, n_heads=4, d_ff=128, dropout=0.0)
    fused = copy.deepcopy(plain)
    fused.prepare_runtime(compute_dtype=torch.float32)
    return plain, fused


def _set_grads(model: torch.nn.Module, grads: list[torch.Tensor]) -> None:
    for p, g in zip(model.parameters(), grads):
        p.grad.copy_(g)  # the fused model's .grad are flat-buffer views: copy, never rebind


def _grads(plain: GPT, seed: int) -> list[torch.Tensor]:
    """Deterministic gradients from the plain model at its CURRENT weights."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, V, (2, 16), generator=g)
    plain.zero_grad(set_to_none=True)
    F.cross_entropy(plain(ids).reshape(-1, V), ids.reshape(-1)).backward()
    return [p.grad.detach().clone() for p in plain.parameters()]


def _roundtrip(sd: dict) -> dict:
    buf = io.BytesIO()
    torch.save(sd, buf)
    buf.seek(0)
    return torch.load(buf, weights_only=True)


def _sync_weights(dst: torch.nn.Module, src: torch.nn.Module) -> None:
    with torch.no_grad():
        for p, q in zip(dst.parameters(), src.parameters()):
            p.copy_(q)


def test_fused_state_dict_has_distinct_step_tensors() -> None:
    _, fused = _models()
    opt = FusedAdamW(fused.parameters(), store=fused.flat_store, lr=1e-3, weight_decay=0.1)
    fused.fused_loss(torch.randint(0, V, (2, 16)), torch.randint(0, V, (2, 16))).backward()
    opt.step()
    sd = _roundtrip(opt.state_dict())
    ptrs = {st["step"].data_ptr() for st in sd["state"].values()}
    assert len(ptrs) == len(sd["state"])
    assert all(float(st["step"]) == 1.0 and st["step"].dtype == torch.float32 for st in sd["state"].values())
    # exporting must not detach the optimizer from its flat moment buffers
    p0 = next(fused.parameters())
    assert opt.state[p0]["exp_avg"].data_ptr() >= opt.exp_avg.data_ptr()


def test_fused_checkpoint_resumes_under_torch_adamw() -> None:
    plain, fused = _models()
    opt_f = FusedAdamW(fused.parameters(), store=fused.flat_store, lr=1e-2, weight_decay=0.1)
    n = 3
    for s in range(n):
        _set_grads(fused, _grads_at(plain, fused, s))
        opt_f.step()
    sd = _roundtrip(opt_f.state_dict())

    torch_model = copy.deepcopy(plain)
    _sync_weights(torch_model, fused)
    opt_t = torch.optim.AdamW(torch_model.parameters(), lr=1e-2, weight_decay=0.1)
    opt_t.load_state_dict(sd)
    for s in range(n, n + 2):
        grads = _grads_at(plain, fused, s)
        _set_grads(fused, grads)
        opt_f.step()
        for p, g in zip(torch_model.parameters(), grads):
            p.grad = g.clone()
        opt_t.step()
    for st in opt_t.state.values():
        assert float(st["step"]) == n + 2
    for p, q in zip(torch_model.parameters(), fused.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), atol=1e-6, rtol=0)


def test_torch_checkpoint_resumes_under_fused_adamw() -> None:
    plain, fused = _models()
    torch_model = copy.deepcopy(plain)
    opt_t = torch.optim.AdamW(torch_model.parameters(), lr=1e-2, weight_decay=0.1)
    n = 3
    for s in range(n):
        grads = _grads_at(plain, torch_model, s)
        for p, g in zip(torch_model.parameters(), grads):
            p.grad = g.clone()
        opt_t.step()
    sd = _roundtrip(opt_t.state_dict())

    _sync_weights(fused, torch_model)
    opt_f = FusedAdamW(fused.parameters(), store=fused.flat_store, lr=1e-2, weight_decay=0.1)
    opt_f.load_state_dict(sd)
    for s in range(n, n + 2):
        grads = _grads_at(plain, torch_model, s)
        _set_grads(fused, grads)
        opt_f.step()
        for p, g in zip(torch_model.parameters(), grads):
            p.grad = g.clone()
        opt_t.step()
    for st in _roundtrip(opt_f.state_dict())["state"].values():
        assert float(st["step"]) == n + 2
    for p, q in zip(torch_model.parameters(), fused.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), atol=1e-6, rtol=0)


def _grads_at(plain: GPT, weights_from: torch.nn.Module, seed: int) -> list[torch.Tensor]:
    _sync_weights(plain, weights_from)
    return _grads(plain, seed)


def _gpt_cfg(tmp_root: str, fused: bool, max_steps: int):  # type: ignore[no-untyped-def]
    from llmtrain.config.schemas import RunConfig

    payload = minimal_payload(
        model={
            "name": "gpt", "vocab_size": 16, "block_size": 8, "d_model": 64, "n_layers": 2, "n_heads": 2,
            "d_ff": 128, "dropout": 0.0, "extra": {"fused": fused},
        },
        trainer={"max_steps": max_steps, "warmup_steps": 0, "micro_batch_size": 2, "grad_accum_steps": 1,
                 "save_every_steps": 3, "eval_every_steps": 100, "log_every_steps": 1, "lr": 1e-2},
        output={"root_dir": tmp_root},
    )
    return RunConfig.model_validate(payload)


def test_trainer_resume_fused_checkpoint_on_module_path(tmp_path) -> None:  # type: ignore[no-untyped-def]
    """Fused-engine run checkpoints at step 3; a module-path (model.extra.fused=false) trainer resumes
    and every per-parameter AdamW step counter reads exactly 5 at the end."""
    from llmtrain.training.trainer import Trainer

    run_a = tmp_path / "a"
    run_a.mkdir()
    tr = Trainer(_gpt_cfg(str(tmp_path), True, 3), run_dir=run_a)
    assert isinstance(tr.optimizer, FusedAdamW)
    tr.fit()
    ckpt = run_a / "checkpoints" / "step_000003.pt"
    assert ckpt.exists()

    run_b = tmp_path / "b"
    run_b.mkdir()
    tb = Trainer(_gpt_cfg(str(tmp_path), False, 5), run_dir=run_b)
    assert isinstance(tb.optimizer, torch.optim.AdamW)
    result = tb.fit(resume_from=str(ckpt))
    assert result.resumed_from_step == 3
    steps = [float(st["step"]) for st in tb.optimizer.state.values()]
    assert steps and all(s == 5.0 for s in steps)
