#!/usr/bin/env python3
"""Trained vs random-init completions and top next-token probabilities (reference notebook
notebooks/trained_vs_random_completion.ipynb), with the KV-cached sampler.

With ``--checkpoint`` it loads a run's newest ``step_*.pt`` (any llmtrain or reference run of the
same config); without one it first trains the config briefly on its synthetic Markov stream so
the comparison is meaningful offline.

    python examples/trained_vs_random_completion.py --config configs/presets/gpt_smoke.yaml --steps 100
"""

from __future__ import annotations

import argparse
import os
import sys
from pathlib import Path

import torch
import yaml

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llmtrain.config.schemas import RunConfig  # noqa: E402
from llmtrain.inference import generate, top_next_tokens  # noqa: E402
from llmtrain.registry import initialize_registries  # noqa: E402
from llmtrain.registry.models import get_model_adapter  # noqa: E402
from llmtrain.training import Trainer  # noqa: E402
from llmtrain.training.checkpoint import CheckpointManager  # noqa: E402


class _IdTokenizer:
    """Space-separated token ids (works for any vocab size, e.g. the 16-token gpt_smoke)."""

    def encode(self, text: str) -> list[int]:
        return [int(t) for t in text.split()]

    def decode(self, ids: list[int]) -> str:
        return " ".join(str(i) for i in ids)


def main(argv: list[str] | None = None) -> dict:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--config", default="configs/presets/gpt_smoke.yaml")
    ap.add_argument("--checkpoint", default=None, help="a step_*.pt file or a checkpoints dir")
    ap.add_argument("--steps", type=int, default=100, help="training steps when no checkpoint is given")
    ap.add_argument("--prompt", default="1 2 3 4", help="space-separated token ids")
    ap.add_argument("--max-new-tokens", type=int, default=8)
    ap.add_argument("--seed", type=int, default=7)
    args = ap.parse_args(argv)

    raw = yaml.safe_load(Path(args.config).read_text())
    raw["mlflow"] = {"enabled": False}
    raw["run"]["device"] = raw["run"].get("device", "cpu")
    raw["trainer"].update({"max_steps": args.steps, "warmup_steps": 0})
    cfg = RunConfig.model_validate(raw)
    initialize_registries()
    adapter = get_model_adapter(cfg.model.name)()
    torch.manual_seed(cfg.run.seed)
    random_model = adapter.build_model(cfg).eval()
    if args.checkpoint:
        path = Path(args.checkpoint)
        path = path if path.is_file() else CheckpointManager(path).latest_checkpoint()
        trained = adapter.build_model(cfg)
        trained.load_state_dict(CheckpointManager(path.parent).load(path)["model_state_dict"])
    else:
        trainer = Trainer(cfg)
        trainer.fit()
        trained = getattr(trainer.model, "module", trainer.model)
    trained = trained.cpu().eval()
    tok = _IdTokenizer()
    prompt = torch.tensor([tok.encode(args.prompt)])
    out = {}
    for name, model in (("trained", trained), ("random", random_model)):
        torch.manual_seed(args.seed)
        ids = generate(model, prompt, args.max_new_tokens, temperature=0.8, top_k=40)
        out[name] = {"completion": tok.decode(ids[0].tolist()), "top_next": top_next_tokens(model, tok, args.prompt, k=5)}
        print(f"=== {name} ===\n{out[name]['completion']}")
        for t, p in out[name]["top_next"]:
            print(f"  {t!r}: {p:.4f}")
    return out


if __name__ == "__main__":
    main()
