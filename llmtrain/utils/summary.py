"""Run summary (JSON dict or "Planned run:" text) — reference ``utils/summary.py:18-217``.

The JSON key set and the text line order are part of the public contract (tests and the
K8s e2e script grep for them), so they are driven from the field tables below.
"""

from __future__ import annotations

import os
from pathlib import Path
from typing import TYPE_CHECKING, Any

from llmtrain.config.schemas import RunConfig
from llmtrain.utils.metadata import DDP_ENV_KEYS

if TYPE_CHECKING:
    from llmtrain.training.trainer import TrainResult

__all__ = ["format_run_summary"]

_SECTION_FIELDS: dict[str, tuple[str, ...]] = {
    "model": (
        "name", "init", "block_size", "d_model", "n_layers", "n_heads", "d_ff", "dropout",
        "tie_embeddings", "vocab_size",
    ),
    "data": (
        "name", "dataset_name", "dataset_config", "text_column", "cache_dir", "num_workers",
        "train_split", "val_split",
    ),
    "trainer": (
        "max_steps", "micro_batch_size", "grad_accum_steps", "lr", "weight_decay",
        "warmup_steps", "max_grad_norm", "log_every_steps", "eval_every_steps",
        "save_every_steps",
    ),
    "ddp": (
        "enabled", "backend", "init_method", "timeout_sec", "find_unused_parameters", "rank",
        "world_size", "local_rank", "master_addr", "master_port",
    ),
    "mlflow": ("enabled", "tracking_uri", "experiment", "run_name", "log_models"),
}
# Fields shown on each text line (the DDP line shows fewer fields plus the env snapshot).
_TEXT_FIELDS: dict[str, tuple[str, ...]] = {
    **_SECTION_FIELDS,
    "ddp": ("enabled", "backend", "init_method", "timeout_sec", "find_unused_parameters"),
}
_TEXT_LABEL = {"model": "Model", "data": "Data", "trainer": "Trainer", "ddp": "DDP", "mlflow": "MLflow"}


def _ddp_env_snapshot() -> dict[str, str | None]:
    return {key: os.environ.get(key) or None for key in DDP_ENV_KEYS}


def _section_values(config: RunConfig, section: str, fields: tuple[str, ...]) -> dict[str, Any]:
    obj = getattr(config, section)
    return {field: getattr(obj, field) for field in fields}


def _training_block(result: TrainResult) -> dict[str, Any]:
    block: dict[str, Any] = {
        "final_step": result.final_step,
        "final_loss": result.final_loss,
        "first_step_loss": result.first_step_loss,
        "total_time": result.total_time,
        "peak_memory": result.peak_memory,
    }
    optional = {
        "parameter_count": result.parameter_count,
        "trainable_parameter_count": result.trainable_parameter_count,
        "final_val_loss": result.final_val_loss,
        "val_metrics": result.val_metrics or None,
        "resumed_from_step": result.resumed_from_step,
    }
    block.update({k: v for k, v in optional.items() if v is not None})
    return block


def format_run_summary(
    *,
    config: RunConfig,
    run_id: str,
    run_dir: str | Path,
    json_output: bool = False,
    resolved_model_adapter: str | None = None,
    resolved_data_module: str | None = None,
    dry_run_steps_executed: int | None = None,
    train_result: TrainResult | None = None,
    resumed_from: str | None = None,
) -> str | dict[str, Any]:
    run_path = Path(run_dir)
    env = _ddp_env_snapshot()

    if json_output:
        summary: dict[str, Any] = {"run_id": run_id, "output_dir": str(run_path)}
        for section, fields in _SECTION_FIELDS.items():
            summary[section] = _section_values(config, section, fields)
        summary["ddp"]["env"] = env
        extras = {
            "resolved_model_adapter": resolved_model_adapter,
            "resolved_data_module": resolved_data_module,
            "dry_run_steps_executed": dry_run_steps_executed,
            "resumed_from": resumed_from,
        }
        summary.update({k: v for k, v in extras.items() if v is not None})
        if train_result is not None:
            summary["training"] = _training_block(train_result)
        return summary

    lines = ["Planned run:", f"  Run ID: {run_id}", f"  Output dir: {run_path}"]
    for section, fields in _TEXT_FIELDS.items():
        values = " ".join(f"{k}={v}" for k, v in _section_values(config, section, fields).items())
        if section == "ddp":
            env_text = ", ".join(f"{k}={v or 'unset'}" for k, v in env.items())
            values += f" env=[{env_text}]"
        lines.append(f"  {_TEXT_LABEL[section]}: {values}")
    if resumed_from is not None:
        lines.append(f"  Resumed from: {resumed_from}")
    if any(v is not None for v in (resolved_model_adapter, resolved_data_module, dry_run_steps_executed)):
        lines.append(
            "  Dry run: "
            f"resolved_model_adapter={resolved_model_adapter} "
            f"resolved_data_module={resolved_data_module} "
            f"steps_executed={dry_run_steps_executed}"
        )
    if train_result is not None:
        r = train_result
        text = f"final_step={r.final_step} final_loss={r.final_loss:.4f} total_time={r.total_time:.2f}s"
        if r.parameter_count is not None:
            text += f" parameter_count={r.parameter_count}"
        if r.trainable_parameter_count is not None:
            text += f" trainable_parameter_count={r.trainable_parameter_count}"
        if r.final_val_loss is not None:
            text += f" final_val_loss={r.final_val_loss:.4f}"
        if r.resumed_from_step is not None:
            text += f" resumed_from_step={r.resumed_from_step}"
        lines.append(f"  Training: {text}")
        if r.val_metrics:
            metrics = " ".join(f"{k}={v:.4f}" for k, v in sorted(r.val_metrics.items()))
            lines.append(f"  Validation: {metrics}")
    return "\n".join(lines)
