#!/usr/bin/env python3
"""One forward/loss pass through the registry-resolved ``dummy_gpt`` adapter and ``dummy_text``
data module (reference notebook notebooks/dummy_plugins_smoke.ipynb, which printed loss 5.107
for an unseeded V=128 model — about ln 128 = 4.85 plus init noise).

    python examples/dummy_plugins_smoke.py
"""

from __future__ import annotations

import os
import sys
from pathlib import Path

import yaml

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llmtrain.config.schemas import RunConfig  # noqa: E402
from llmtrain.registry import initialize_registries  # noqa: E402
from llmtrain.registry.data import get_data_module  # noqa: E402
from llmtrain.registry.models import get_model_adapter  # noqa: E402

ROOT = Path(__file__).resolve().parents[1]


def main() -> float:
    cfg = RunConfig.model_validate(yaml.safe_load((ROOT / "configs/presets/example.yaml").read_text()))
    cfg = cfg.model_copy(update={
        "model": cfg.model.model_copy(update={"name": "dummy_gpt", "vocab_size": 128, "d_model": 64, "block_size": 32}),
        "data": cfg.data.model_copy(update={"name": "dummy_text", "num_workers": 0}),
        "trainer": cfg.trainer.model_copy(update={"max_steps": 3, "micro_batch_size": 2}),
    })
    initialize_registries()
    adapter = get_model_adapter("dummy_gpt")()
    data = get_data_module("dummy_text")()
    model = adapter.build_model(cfg)
    data.setup(cfg, tokenizer=adapter.build_tokenizer(cfg))
    batch = next(iter(data.train_dataloader()))
    loss, metrics = adapter.compute_loss(model, batch)
    print("loss:", float(loss))
    print("metrics:", {k: float(v) for k, v in metrics.items()})
    return float(loss)


if __name__ == "__main__":
    main()
