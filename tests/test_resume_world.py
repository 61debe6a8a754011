"""Resume under data parallelism (real 2-process gloo worlds on CPU): an interrupted and resumed
2-rank run with dropout equals the uninterrupted one bit for bit (each rank's own RNG streams are
in the checkpoint), and a 2-rank checkpoint resumed on ONE process continues after the global
samples already trained on, with a warning (reference trainer.py:336-347 gives up on replay
under DDP)."""

from __future__ import annotations

import logging
import os
import socket
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from llmtrain.config.schemas import RunConfig

from conftest import minimal_payload


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cfg(**ddp) -> RunConfig:  # type: ignore[no-untyped-def]
    model = {"name": "gpt", "vocab_size": 32, "block_size": 8, "d_model": 64, "n_layers": 1, "n_heads": 2,
             "d_ff": 64, "dropout": 0.2, "extra": {"fused": True}}
    return RunConfig.model_validate(minimal_payload(
        model=model, data={"name": "synthetic_tokens", "num_workers": 0,
                           "extra": {"train_sequences": 64, "val_sequences": 0}},
        ddp={"enabled": True, **ddp}, run={"name": "w", "seed": 5},
        trainer={"max_steps": 4, "warmup_steps": 0, "micro_batch_size": 2, "grad_accum_steps": 1,
                 "save_every_steps": 2, "log_every_steps": 2, "eval_every_steps": 100},
    ))


def _worker(rank: int, world: int, port: int, out_dir: str) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    from llmtrain.parallel.dist import DDPState
    from llmtrain.training.trainer import Trainer

    state = DDPState(rank=rank, world_size=world, local_rank=rank, is_main=rank == 0)
    out = Path(out_dir)
    cfg = _cfg()
    full = Trainer(cfg, run_dir=out / "full" if rank == 0 else None, ddp_state=state)
    full.fit()
    part = Trainer(cfg, run_dir=out / "part" if rank == 0 else None, ddp_state=state)
    part.fit(max_steps_override=2)  # checkpoint at step 2, same LR horizon (max_steps 4)
    dist.barrier()
    resumed = Trainer(cfg, run_dir=out / "resumed" if rank == 0 else None, ddp_state=state)
    resumed.fit(resume_from=str(out / "part" / "checkpoints"))
    torch.save({"full": full.model.module.flat_store.master.clone(),
                "resumed": resumed.model.module.flat_store.master.clone()}, out / f"r{rank}.pt")
    dist.destroy_process_group()


def test_ddp_resume_is_exact_and_world_change_continues(
    tmp_path: Path, trainer_records: list[logging.LogRecord]
) -> None:
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for rank in (0, 1):
        r = torch.load(tmp_path / f"r{rank}.pt", weights_only=True)
        assert torch.equal(r["full"], r["resumed"]), f"rank {rank}: resumed run differs"

    # the 2-rank checkpoint at step 2 on ONE process: global samples 0..7 were trained on
    # (2 steps x micro-batch 2 x 2 ranks), so this process starts at its batch 4 = samples 8, 9
    from llmtrain.training.trainer import Trainer

    cfg = RunConfig.model_validate({**_cfg().model_dump(), "ddp": {"enabled": False}})
    trainer = Trainer(cfg)
    seen: list[torch.Tensor] = []
    adapter = trainer._adapter
    original = adapter.compute_loss

    def spy(model, batch):  # type: ignore[no-untyped-def]
        seen.append(batch["input_ids"].clone())
        return original(model, batch)

    adapter.compute_loss = spy  # type: ignore[method-assign]
    trainer.fit(max_steps_override=3, resume_from=str(tmp_path / "part" / "checkpoints"))
    data = trainer._train_loader.dataset
    want = torch.stack([data[8]["input_ids"], data[9]["input_ids"]])
    assert torch.equal(seen[0], want)
    text = " ".join(r.getMessage() for r in trainer_records)
    assert "saved at world_size=2, resuming at world_size=1" in text and "global sample 8" in text


@pytest.mark.parametrize("value", [0, 1])
def test_replay_without_record_falls_back(value: int) -> None:  # noqa: ARG001 - two identical cases
    from llmtrain.training.trainer import Trainer

    cfg = RunConfig.model_validate({**_cfg().model_dump(), "ddp": {"enabled": False}})
    tr = Trainer(cfg)
    payload = {"config": cfg.model_dump()}
    assert tr._replay_batches(payload, 3) == 3  # step x grad_accum
    payload["llmtrain_extra"] = {"world_size": 1, "batches_consumed": 7}
    assert tr._replay_batches(payload, 3) == 7
