"""hipGraph-captured optimizer steps (``trainer.extra.cuda_graph``, llmtrain.training.graph_step) on
an MI355X: the replayed step trains exactly like the eager one — same per-step losses and grad
norms, same final weights and AdamW state, with a warm-up learning-rate schedule (the per-step
AdamW scalars are staged, not baked into the graph) and gradient accumulation — and it really
replays (one capture, every later step a replay).  Also: checkpoint + resume from a graphed run."""

from __future__ import annotations

import pytest
import torch

from llmtrain.config.schemas import RunConfig

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("gpu_device")]


def _cfg(root: str, graph: bool, *, max_steps: int = 10, save_every: int = 100, dropout: float = 0.0,
         warmup: int = 2) -> RunConfig:
    return RunConfig.model_validate({
        "schema_version": 1,
        "run": {"name": "gpu-graph", "device": "cuda", "precision": "bf16", "seed": 11, "deterministic": True},
        "model": {"name": "gpt", "vocab_size": 512, "block_size": 128, "d_model": 128, "n_layers": 2,
                  "n_heads": 2, "d_ff": 512, "dropout": dropout},
        "data": {"name": "synthetic_tokens", "num_workers": 0, "extra": {"train_sequences": 256, "val_sequences": 16}},
        "trainer": {"max_steps": max_steps, "micro_batch_size": 8, "grad_accum_steps": 2, "lr": 2e-3,
                    "warmup_steps": 4, "log_every_steps": 2, "eval_every_steps": 100, "save_every_steps": save_every,
                    "extra": {"cuda_graph": graph, "cuda_graph_warmup": warmup}},
        "ddp": {}, "mlflow": {"enabled": False}, "logging": {"log_to_file": False},
        "output": {"root_dir": root},
    })


def _run(trainer, steps: int) -> tuple[list[float], list[float]]:
    batches = trainer.batch_stream()
    losses, norms = [], []
    for _ in range(steps):
        loss, _ = trainer.train_step(batches)
        losses.append(float(loss))
        norms.append(float(trainer.last_grad_norm))
    torch.cuda.synchronize()
    return losses, norms


def test_graphed_steps_match_eager(tmp_path) -> None:
    from llmtrain.training.trainer import Trainer

    eager = Trainer(_cfg(str(tmp_path / "e"), False))
    graphed = Trainer(_cfg(str(tmp_path / "g"), True))
    steps = 10
    le, ne = _run(eager, steps)
    lg, ng = _run(graphed, steps)
    g = graphed._graphed
    assert g is not None and g.eager_steps == 2 and g.replays == steps - 2
    print("eager", le, "\ngraph", lg)
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-6 * abs(a), (le, lg)
    for a, b in zip(ne, ng):
        assert abs(a - b) <= 1e-5 * abs(a), (ne, ng)
    se, sg = eager.model.engine.store, graphed.model.engine.store
    assert torch.allclose(se.master, sg.master, rtol=0, atol=1e-6)
    oe, og = eager._optimizer, graphed._optimizer
    assert oe.steps_taken == og.steps_taken == steps
    assert torch.allclose(oe.exp_avg_sq, og.exp_avg_sq, rtol=1e-5, atol=1e-12)
    assert eager._optimizer.param_groups[0]["lr"] == graphed._optimizer.param_groups[0]["lr"]


def test_graphed_dropout_matches_eager_staging(tmp_path) -> None:
    """Dropout under a captured step: replays get fresh masks from the restaged seed word, and
    they are exactly the masks the same mode's eager steps draw (a run whose every step is eager
    — warm-up longer than the run — trains identically)."""
    from llmtrain.training.trainer import Trainer

    eager = Trainer(_cfg(str(tmp_path / "e"), True, dropout=0.1, warmup=100))
    graphed = Trainer(_cfg(str(tmp_path / "g"), True, dropout=0.1))
    le, _ = _run(eager, 8)
    lg, _ = _run(graphed, 8)
    assert eager._graphed.replays == 0 and graphed._graphed.replays == 6
    for a, b in zip(le, lg):
        assert abs(a - b) <= 1e-6 * abs(a), (le, lg)
    assert torch.allclose(eager.model.engine.store.master, graphed.model.engine.store.master, rtol=0, atol=1e-6)


@pytest.mark.parametrize("dropout", [0.0, 0.1])
def test_graphed_fit_checkpoint_resume(tmp_path, dropout) -> None:
    """fit() with a captured step, a checkpoint at step 6, and a graphed resume to step 10 that
    ends where the uninterrupted graphed run ends (deterministic kernels: 1e-5, the reference's
    resume tolerance) — with dropout too: the masks depend on (run seed, step), not on RNG history."""
    from llmtrain.training.trainer import Trainer

    full = Trainer(_cfg(str(tmp_path / "a"), True, dropout=dropout), run_dir=tmp_path / "a" / "run").fit()
    part = tmp_path / "b" / "run"
    Trainer(_cfg(str(tmp_path / "b"), True, save_every=3, dropout=dropout), run_dir=part).fit(max_steps_override=6)
    resumed = Trainer(_cfg(str(tmp_path / "b"), True, dropout=dropout), run_dir=tmp_path / "b" / "run2").fit(
        resume_from=str(part / "checkpoints")
    )
    assert resumed.resumed_from_step == 6 and resumed.final_step == 10
    assert abs(resumed.final_loss - full.final_loss) <= 1e-5 * abs(full.final_loss)


def test_graphed_padded_batch_runs_eagerly(tmp_path) -> None:
    """A batch carrying a padding mask does not fit the captured graph: that step runs eagerly
    (through the key-padding attention path), and the following full batches replay again."""
    import math

    from llmtrain.training.trainer import Trainer

    trainer = Trainer(_cfg(str(tmp_path / "p"), True))
    batches = trainer.batch_stream()
    for _ in range(4):  # 2 eager warm-up steps, the capture step, one replay
        trainer.train_step(batches)
    g = trainer._graphed
    assert g is not None and g.replays == 2 and g.eager_steps == 2

    class _Padded:
        def next(self):
            b = dict(batches.next())
            mask = torch.ones_like(b["input_ids"])
            mask[:, -5:] = 0
            b["attention_mask"] = mask
            return b

    loss, _ = trainer.train_step(_Padded())
    assert g.replays == 2 and g.eager_steps == 3 and math.isfinite(float(loss))
    loss, _ = trainer.train_step(batches)
    assert g.replays == 3 and math.isfinite(float(loss))
