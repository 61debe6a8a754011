"""Strict, frozen Pydantic schema for an ``llmtrain`` run.

Contract parity with the reference schema (``src/llmtrain/config/schemas.py:8-186``):
every section and every field/default of the reference exists here, so the reference presets
validate unchanged.  The MI355X build *widens* a few literals instead of renaming them:

* ``run.device`` accepts ``"cuda"`` (PyTorch-ROCm's device type for HIP GPUs) and ``"rocm"``
  (alias) in addition to ``"cpu"``/``"mps"``.
* ``ddp.backend`` accepts ``"nccl"`` (RCCL on ROCm) and ``"rccl"`` (alias) next to ``"gloo"``.
* ``run.precision`` (new, default ``"fp32"`` = reference numerics) selects bf16 compute on GPU.

New knobs that are not part of the reference contract live in the existing free-form
``extra`` bags (``model.extra``, ``trainer.extra``, ``data.extra``) and in one new bag,
``ddp.extra`` (the startup transport checks of :mod:`llmtrain.parallel.comm`).
"""

from __future__ import annotations

from typing import Any, Literal

from pydantic import BaseModel, ConfigDict, Field, model_validator

__all__ = [
    "DataConfig",
    "DDPConfig",
    "LoggingConfig",
    "MLflowConfig",
    "ModelConfig",
    "OutputConfig",
    "RunConfig",
    "RunSectionConfig",
    "TrainerConfig",
]

_STRICT = ConfigDict(extra="forbid", frozen=True, validate_default=True)


class _Section(BaseModel):
    """Base for every config section: unknown keys rejected, instances immutable."""

    model_config = _STRICT


class RunSectionConfig(_Section):
    """Run identity, seeding and placement."""

    name: str
    seed: int = 1337
    device: Literal["cpu", "mps", "cuda", "rocm"] = "cpu"
    deterministic: bool = True
    notes: str | None = None
    precision: Literal["fp32", "bf16"] = "fp32"


class ModelConfig(_Section):
    """Architecture hyper-parameters consumed by model adapters."""

    name: str
    init: Literal["random"] = "random"
    block_size: int = Field(256, ge=8)
    d_model: int = Field(384, ge=64)
    n_layers: int = Field(6, ge=1)
    n_heads: int = Field(6, ge=1)
    d_ff: int = Field(1536, ge=64)
    dropout: float = Field(0.1, ge=0.0, lt=1.0)
    tie_embeddings: bool = True
    vocab_size: int | None = None
    extra: dict[str, Any] = Field(default_factory=dict)

    @model_validator(mode="after")
    def _check_shapes(self) -> ModelConfig:
        if self.d_model % self.n_heads:
            raise ValueError("d_model must be divisible by n_heads")
        if self.d_ff < self.d_model:
            raise ValueError("d_ff must be greater than or equal to d_model")
        return self


class DataConfig(_Section):
    """Data module selection plus optional Hugging Face dataset coordinates."""

    name: str
    cache_dir: str = ".cache/datasets"
    num_workers: int = Field(2, ge=0)
    train_split: str = "train"
    val_split: str = "validation"
    dataset_name: str | None = None
    dataset_config: str | None = None
    text_column: str | None = None
    extra: dict[str, Any] = Field(default_factory=dict)


class TrainerConfig(_Section):
    """Optimizer-step loop pacing."""

    max_steps: int = Field(1000, ge=1)
    micro_batch_size: int = Field(8, ge=1)
    grad_accum_steps: int = Field(4, ge=1)
    lr: float = Field(3e-4, gt=0.0)
    weight_decay: float = Field(0.1, ge=0.0)
    warmup_steps: int = Field(100, ge=0)
    max_grad_norm: float = Field(1.0, gt=0.0)
    log_every_steps: int = Field(10, ge=1)
    eval_every_steps: int = Field(100, ge=1)
    save_every_steps: int = Field(500, ge=1)
    extra: dict[str, Any] = Field(default_factory=dict)

    @model_validator(mode="after")
    def _check_warmup(self) -> TrainerConfig:
        if self.warmup_steps > self.max_steps:
            raise ValueError("warmup_steps cannot exceed max_steps")
        return self


class DDPConfig(_Section):
    """Data-parallel runtime; env vars (torchrun / K8s entrypoint) take precedence."""

    enabled: bool = False
    backend: Literal["gloo", "nccl", "rccl"] = "gloo"
    init_method: Literal["env://"] = "env://"
    timeout_sec: int = Field(1800, ge=1)
    find_unused_parameters: bool = False
    rank: int | None = None
    world_size: int | None = None
    local_rank: int | None = None
    master_addr: str | None = None
    master_port: int | None = None
    # MI355X additions (llmtrain.parallel.comm): probe_allreduce_mib, probe_iters, min_busbw_gbps,
    # log_transport, transport_log_dir, max_channels, min_channels
    extra: dict[str, Any] = Field(default_factory=dict)


class MLflowConfig(_Section):
    """Experiment tracking (rank 0 only)."""

    enabled: bool = True
    tracking_uri: str = "file:./mlruns"
    experiment: str = "llm-train-k8s"
    run_name: str | None = None
    log_models: bool = False


class LoggingConfig(_Section):
    """stdout / file logging."""

    level: Literal["DEBUG", "INFO", "WARNING", "ERROR"] = "INFO"
    json_output: bool = True
    log_to_file: bool = True
    file_name: str = "train.log"


class OutputConfig(_Section):
    """Run directory placement and persistence toggles."""

    root_dir: str = "runs"
    run_id: str | None = None
    save_config_copy: bool = True
    save_meta_json: bool = True


class RunConfig(_Section):
    """The whole run. All nine sections are required keys (each may be ``{}``)."""

    schema_version: int = Field(1, ge=1)
    run: RunSectionConfig
    model: ModelConfig
    data: DataConfig
    trainer: TrainerConfig
    ddp: DDPConfig
    mlflow: MLflowConfig
    logging: LoggingConfig
    output: OutputConfig
