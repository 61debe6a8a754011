"""Non-finite gradient guard (the reference clips, steps and saves unconditionally,
reference ``training/trainer.py:390-413``): a NaN gradient injected at one step is skipped — no
weight or moment is touched — the run completes, no checkpoint holds a non-finite tensor, and a
``--resume`` from the newest checkpoint reproduces the uninterrupted run bit for bit.  Both the
fused engine (CPU reference ops, the same skip contract as the HIP kernel) and the module path
(torch AdamW + ``clip_grad_norm_``) are covered, plus a 2-rank gloo world where only one rank's
backward is poisoned (the all-reduce spreads it, every rank skips the same step)."""

from __future__ import annotations

import math
import os
import socket
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from llmtrain import ops
from llmtrain.config.schemas import RunConfig
from llmtrain.training.trainer import Trainer

from conftest import minimal_payload


def _cfg(  # type: ignore[no-untyped-def]
    fused: bool, *, inject: int | None = 3, max_steps: int = 6, ddp: bool = False, **extra
) -> RunConfig:
    model = {"name": "gpt", "vocab_size": 32, "block_size": 8, "d_model": 64, "n_layers": 1, "n_heads": 2,
             "d_ff": 64, "dropout": 0.0, "extra": {"fused": fused}}
    trainer_extra = dict(extra)
    if inject is not None:
        trainer_extra["inject_nonfinite_grad_at_step"] = inject
    return RunConfig.model_validate(minimal_payload(
        model=model, data={"name": "synthetic_tokens", "num_workers": 0,
                           "extra": {"train_sequences": 64, "val_sequences": 0}},
        ddp={"enabled": ddp}, run={"name": "nf", "seed": 3},
        trainer={"max_steps": max_steps, "warmup_steps": 0, "micro_batch_size": 2, "grad_accum_steps": 2,
                 "save_every_steps": 2, "log_every_steps": 1, "eval_every_steps": 100, "lr": 1e-2,
                 "extra": trainer_extra},
    ))


def _weights(trainer: Trainer) -> torch.Tensor:
    return torch.cat([p.detach().reshape(-1).float() for p in trainer._raw_model.parameters()])


def test_clip_coef_is_nan_for_nonfinite_norm() -> None:
    for bad in (float("nan"), float("inf")):
        out = ops.clip_coef(torch.tensor(bad), 1.0)
        assert math.isnan(float(out[1])), bad
    out = ops.clip_coef(torch.tensor(16.0), 1.0)
    assert float(out[0]) == 4.0 and abs(float(out[1]) - 1.0 / (4.0 + 1e-6)) < 1e-7
    assert float(ops.clip_coef(torch.tensor(0.25), 1.0)[1]) == 1.0


def test_adamw_flat_skips_and_counts() -> None:
    n = 37
    p = torch.randn(n)
    g, m, v = torch.randn(n), torch.randn(n).abs(), torch.randn(n).abs()
    before = [t.clone() for t in (p, m, v)]
    skipped = torch.zeros(2, dtype=torch.int32)
    kw = dict(lr=1e-2, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.1, step=3)
    for _ in range(2):
        ops.adamw_flat(p, g, m, v, None, grad_scale=torch.tensor(float("nan")), skipped=skipped, **kw)
    assert all(torch.equal(a, b) for a, b in zip((p, m, v), before))
    assert skipped.tolist() == [2, 2]
    ops.adamw_flat(p, g, m, v, None, grad_scale=torch.tensor(1.0), skipped=skipped, **kw)
    assert not torch.equal(p, before[0])
    assert skipped.tolist() == [2, 0]


@pytest.mark.parametrize("fused", [True, False], ids=["fused", "module"])
def test_injected_nan_step_is_skipped_and_resume_is_exact(tmp_path: Path, fused: bool) -> None:
    cfg = _cfg(fused)
    full = Trainer(cfg, run_dir=tmp_path / "full")
    result = full.fit()
    assert math.isfinite(result.final_loss)
    assert full.skipped_steps() == (1, 0)
    w_full = _weights(full)
    assert bool(torch.isfinite(w_full).all())

    ckpts = sorted((tmp_path / "full" / "checkpoints").glob("step_*.pt"))
    assert [c.stem for c in ckpts] == ["step_000002", "step_000004", "step_000006"]
    for c in ckpts:
        payload = torch.load(c, weights_only=False)
        tensors = list(payload["model_state_dict"].values())
        for st in payload["optimizer_state_dict"]["state"].values():
            tensors += [t for t in st.values() if isinstance(t, torch.Tensor)]
        assert all(bool(torch.isfinite(t.float()).all()) for t in tensors), c.name

    # the skipped step left the weights exactly where the step before had put them
    upto2 = Trainer(cfg)
    upto2.fit(max_steps_override=2)
    upto3 = Trainer(cfg)
    upto3.fit(max_steps_override=3)
    assert torch.equal(_weights(upto2), _weights(upto3))

    # an interrupted run (checkpoint at step 2, before the injected step) resumed from its newest
    # checkpoint replays the skip and ends bitwise equal to the uninterrupted run
    part = Trainer(cfg, run_dir=tmp_path / "part")
    part.fit(max_steps_override=2)
    resumed = Trainer(cfg, run_dir=tmp_path / "resumed")
    resumed.fit(resume_from=str(tmp_path / "part" / "checkpoints"))
    assert torch.equal(_weights(resumed), w_full)
    # and from the step-4 checkpoint of the full run (after the skip)
    again = Trainer(cfg, run_dir=tmp_path / "again")
    again.fit(resume_from=str(tmp_path / "full" / "checkpoints" / "step_000004.pt"))
    assert torch.equal(_weights(again), w_full)


def test_consecutive_skips_raise(tmp_path: Path) -> None:
    cfg = _cfg(True, inject=2, max_skipped_steps=1)
    trainer = Trainer(cfg, run_dir=tmp_path / "r")
    with pytest.raises(FloatingPointError, match="consecutive optimizer steps skipped"):
        trainer.fit()


def test_checkpoint_refused_for_nonfinite_state(tmp_path: Path) -> None:
    cfg = _cfg(True, inject=None, halt_on_nan=False)
    trainer = Trainer(cfg, run_dir=tmp_path / "r")
    store = trainer._raw_model.flat_store
    trainer.fit(max_steps_override=1)
    store.master[0] = float("nan")  # weights poisoned by something other than a gradient
    with pytest.raises(FloatingPointError, match="refusing to checkpoint"):
        trainer.fit(max_steps_override=2)
    assert not (tmp_path / "r" / "checkpoints" / "step_000002.pt").exists()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, out_dir: str) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from llmtrain.parallel.dist import DDPState

    state = DDPState(rank=rank, world_size=world, local_rank=rank, is_main=rank == 0)
    out = Path(out_dir)
    for fused in (True, False):
        cfg = _cfg(fused, ddp=True, max_steps=4, inject_nonfinite_rank=1)
        trainer = Trainer(cfg, run_dir=out / f"f{int(fused)}" if rank == 0 else None, ddp_state=state)
        trainer.fit()
        torch.save({"w": _weights(trainer), "skipped": list(trainer.skipped_steps())}, out / f"r{rank}_{int(fused)}.pt")
    dist.destroy_process_group()


def test_ddp_one_rank_poisoned_every_rank_skips(tmp_path: Path) -> None:
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for fused in (0, 1):
        r0 = torch.load(tmp_path / f"r0_{fused}.pt", weights_only=True)
        r1 = torch.load(tmp_path / f"r1_{fused}.pt", weights_only=True)
        assert r0["skipped"] == r1["skipped"] == [1, 0]
        assert torch.equal(r0["w"], r1["w"]) and bool(torch.isfinite(r0["w"]).all())
