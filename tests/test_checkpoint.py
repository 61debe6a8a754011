"""Checkpoint format, pruning, resume and resume parity (reference tests/test_checkpoint.py),
plus atomic writes, safe loading of reference-style payloads and the fused path."""

from __future__ import annotations

import random
from pathlib import Path

import numpy as np
import pytest
import torch

from llmtrain.config.schemas import RunConfig
from llmtrain.training.checkpoint import REQUIRED_KEYS, CheckpointManager
from llmtrain.training.trainer import Trainer

from conftest import minimal_payload


def _cfg(tmp: Path, fused: bool | None = None, **trainer) -> RunConfig:  # type: ignore[no-untyped-def]
    t = {"max_steps": 6, "warmup_steps": 0, "micro_batch_size": 2, "grad_accum_steps": 1, "save_every_steps": 2,
         "log_every_steps": 2, "eval_every_steps": 100}
    t.update(trainer)
    over: dict = {"trainer": t, "output": {"root_dir": str(tmp / "runs")}}
    if fused is not None:
        over["model"] = {"name": "gpt", "vocab_size": 32, "block_size": 8, "d_model": 64, "n_layers": 1,
                         "n_heads": 2, "d_ff": 64, "dropout": 0.0, "extra": {"fused": fused}}
    return RunConfig.model_validate(minimal_payload(**over))


def test_save_layout_keys_and_rng(tmp_path: Path) -> None:
    run_dir = tmp_path / "run"
    Trainer(_cfg(tmp_path, max_steps=2), run_dir=run_dir).fit()
    path = run_dir / "checkpoints" / "step_000002.pt"
    assert path.exists() and not list(path.parent.glob("*.tmp"))
    payload = CheckpointManager(path.parent).load(path)
    assert REQUIRED_KEYS <= set(payload)
    assert set(payload["rng_states"]) >= {"python", "numpy", "torch"}
    assert payload["step"] == 2 and payload["config"]["trainer"]["max_steps"] == 2
    state = payload["optimizer_state_dict"]["state"][0]
    assert set(state) == {"step", "exp_avg", "exp_avg_sq"}


def test_pruning_and_latest(tmp_path: Path) -> None:
    run_dir = tmp_path / "run"
    Trainer(_cfg(tmp_path, max_steps=9, extra={"keep_last_k": 2}), run_dir=run_dir).fit()
    mgr = CheckpointManager(run_dir / "checkpoints")
    names = [p.name for p in mgr.checkpoints()]
    assert names == ["step_000008.pt", "step_000009.pt"]  # save every 2 + final step, keep 2
    assert mgr.latest_checkpoint().name == "step_000009.pt"
    (run_dir / "checkpoints" / "step_000010.pt").write_bytes(b"")
    assert mgr.latest_checkpoint().name == "step_000010.pt"  # numeric sort


def test_load_rejects_missing_keys(tmp_path: Path) -> None:
    bad = tmp_path / "step_000001.pt"
    torch.save({"step": 1}, bad)
    with pytest.raises(ValueError, match="missing keys"):
        CheckpointManager(tmp_path).load(bad)


def test_reference_style_numpy_rng_loads_safely(tmp_path: Path) -> None:
    payload = {k: {} for k in REQUIRED_KEYS}
    payload["step"] = 3
    payload["rng_states"] = {"python": random.getstate(), "numpy": np.random.get_state(),
                             "torch": torch.random.get_rng_state()}
    path = tmp_path / "step_000003.pt"
    torch.save(payload, path)
    loaded = CheckpointManager(tmp_path).load(path)
    assert isinstance(loaded["rng_states"]["numpy"][1], np.ndarray)


@pytest.mark.parametrize("fused", [None, True])
def test_resume_parity(tmp_path: Path, fused) -> None:  # type: ignore[no-untyped-def]
    torch.use_deterministic_algorithms(True)
    try:
        full = Trainer(_cfg(tmp_path / "a", fused=fused, max_steps=6), run_dir=tmp_path / "a" / "run").fit()
        part_dir = tmp_path / "b" / "run"
        Trainer(_cfg(tmp_path / "b", fused=fused, max_steps=6), run_dir=part_dir).fit(max_steps_override=4)
        resumed = Trainer(_cfg(tmp_path / "b", fused=fused, max_steps=6), run_dir=tmp_path / "b" / "run2").fit(
            resume_from=str(part_dir / "checkpoints")
        )
    finally:
        torch.use_deterministic_algorithms(False)
    assert resumed.resumed_from_step == 4 and resumed.first_step_loss is None
    assert abs(resumed.final_loss - full.final_loss) <= 1e-5


def test_resume_by_file_and_run_id_and_errors(tmp_path: Path, monkeypatch: pytest.MonkeyPatch) -> None:
    cfg = _cfg(tmp_path, max_steps=4)
    runs = Path(cfg.output.root_dir)
    Trainer(cfg, run_dir=runs / "rid").fit()
    ckpt = runs / "rid" / "checkpoints" / "step_000004.pt"
    t = Trainer(cfg)
    assert t._resolve_resume_path(str(ckpt)) == ckpt
    assert t._resolve_resume_path("rid") == ckpt
    with pytest.raises(FileNotFoundError):
        t._resolve_resume_path(str(tmp_path / "nope.pt"))
    with pytest.raises(FileNotFoundError):
        t._resolve_resume_path("unknown_run")
    result = Trainer(_cfg(tmp_path, max_steps=4)).fit(resume_from=str(ckpt))
    assert result.resumed_from_step == 4 and result.final_step == 4


def test_config_mismatch_warns(tmp_path: Path, trainer_records) -> None:  # type: ignore[no-untyped-def]
    cfg = _cfg(tmp_path, max_steps=2)
    Trainer(cfg, run_dir=tmp_path / "run").fit()
    other = _cfg(tmp_path, max_steps=3, lr=1e-3)
    Trainer(other).fit(resume_from=str(tmp_path / "run" / "checkpoints"))
    assert any("config mismatch" in r.getMessage() for r in trainer_records)


def test_async_writer_matches_sync_and_flushes(tmp_path) -> None:
    """The background writer produces the same file contents as the synchronous path, keeps the
    tied-weight aliasing, writes atomically, prunes, and wait() re-raises a write error."""
    import torch

    from llmtrain.training.checkpoint import CheckpointManager

    class _Sched:
        def state_dict(self):
            return {"last_epoch": 3}

    class _Cfg:
        def model_dump(self):
            return {"x": 1}

    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 4))
    model[1].weight = model[0].weight  # tied, like lm_head / token_embedding
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    model(torch.randn(2, 4)).sum().backward()
    opt.step()
    sync = CheckpointManager(tmp_path / "sync", keep_last_k=1)
    asyn = CheckpointManager(tmp_path / "async", keep_last_k=1, async_write=True)
    for step in (1, 2):
        sync.save(step, model, opt, _Sched(), _Cfg())
        asyn.save(step, model, opt, _Sched(), _Cfg())
    asyn.wait()
    assert [p.name for p in asyn.checkpoints()] == ["step_000002.pt"]
    assert not list((tmp_path / "async").glob("*.tmp"))
    a, b = sync.load(sync.latest_checkpoint()), asyn.load(asyn.latest_checkpoint())
    for k, v in a["model_state_dict"].items():
        assert torch.equal(v, b["model_state_dict"][k])
    sd = b["model_state_dict"]
    assert sd["0.weight"].untyped_storage().data_ptr() == sd["1.weight"].untyped_storage().data_ptr()
    assert a["optimizer_state_dict"]["state"][0]["step"] == b["optimizer_state_dict"]["state"][0]["step"]

    bad = CheckpointManager(tmp_path / "bad", async_write=True)
    bad._write = lambda payload, path: (_ for _ in ()).throw(OSError("disk full"))  # type: ignore[method-assign]
    bad.save(1, model, opt, _Sched(), _Cfg())
    try:
        bad.wait()
    except OSError as exc:
        assert "disk full" in str(exc)
    else:
        raise AssertionError("wait() must re-raise the background write error")


def test_async_snapshot_is_taken_at_save_time(tmp_path) -> None:
    """Parameters changed right after save() (the next optimizer step) do not leak into the file
    the background thread is still writing."""
    import torch

    from llmtrain.training.checkpoint import CheckpointManager

    class _Sched:
        def state_dict(self):
            return {}

    class _Cfg:
        def model_dump(self):
            return {}

    model = torch.nn.Linear(8, 8)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    before = model.weight.detach().clone()
    mgr = CheckpointManager(tmp_path, async_write=True)
    mgr.save(1, model, opt, _Sched(), _Cfg())
    with torch.no_grad():
        model.weight.add_(1.0)
    mgr.wait()
    assert torch.equal(mgr.load(mgr.latest_checkpoint())["model_state_dict"]["weight"], before)
