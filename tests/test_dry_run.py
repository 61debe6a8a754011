"""Dry run (reference tests/test_dry_run.py)."""

from __future__ import annotations

import torch
from torch.utils.data import DataLoader

from llmtrain.config.schemas import RunConfig
from llmtrain.data.base import DataModule
from llmtrain.registry.data import DATA_MODULES, register_data_module
from llmtrain.training.dry_run import run_dry_run

from conftest import minimal_payload


def test_dry_run_executes_five_steps() -> None:
    result = run_dry_run(RunConfig.model_validate(minimal_payload(trainer={"max_steps": 20, "warmup_steps": 0})))
    assert result.steps_executed == 5 and result.resolved_data_module == "dummy_text"


def test_dry_run_capped_by_max_steps_and_short_loader() -> None:
    assert run_dry_run(RunConfig.model_validate(minimal_payload(trainer={"max_steps": 2, "warmup_steps": 0}))).steps_executed == 2

    @register_data_module("short_tmp")
    class Short(DataModule):
        def setup(self, cfg, tokenizer=None):  # type: ignore[no-untyped-def]
            self.ds = [{"input_ids": torch.zeros(4, dtype=torch.long), "labels": torch.zeros(4, dtype=torch.long)}] * 2

        def train_dataloader(self):  # type: ignore[no-untyped-def]
            return DataLoader(self.ds, batch_size=1)

        def val_dataloader(self):  # type: ignore[no-untyped-def]
            return None

    try:
        cfg = RunConfig.model_validate(minimal_payload(data={"name": "short_tmp"}, trainer={"max_steps": 10, "warmup_steps": 0}))
        assert run_dry_run(cfg).steps_executed == 2
    finally:
        DATA_MODULES.unregister("short_tmp")
