"""Optimizer-step training loop (reference ``training/trainer.py:30-548``), MI355X build.

Loop semantics kept from the reference: ``grad_accum_steps`` micro-batches per optimizer step
(communication skipped on all but the last), global-norm clipping, AdamW, a LambdaLR with
linear warm-up then cosine decay to 0 at ``max_steps`` (step 0 uses lr=0 when warm-up > 0),
rank-0 checkpointing BEFORE evaluation, interval metrics every ``log_every_steps`` and at the
final step, token-weighted evaluation every ``eval_every_steps`` and at the final step, and
``--resume`` from a run id, checkpoint directory or ``step_N.pt``.

What changes on the MI355X path:

* the fused GPT engine + flat-buffer gradient reducer + fused AdamW (one kernel, clip
  coefficient read on device) replace autograd/DDP/foreach-AdamW when the model supports it;
* the loss is accumulated ON DEVICE; the host reads it once per log interval (the reference
  calls ``.item()`` on every micro-step — a pipeline-draining sync);
* metric collectives use device tensors (RCCL cannot reduce CPU tensors);
* resume replays the data order on every rank (each rank skips its own shard's batches — the
  reference disables replay under DDP);
* ``peak_memory`` reports ``torch.cuda.max_memory_allocated`` (GiB) on GPU;
* optional ``trainer.extra``: ``keep_last_k``, ``fail_at_step`` / ``fail_rank`` (fault injection:
  that rank raises at that step of a run that did not resume — one simulated crash per job),
  ``profile`` (torch.profiler window), ``bucket_cap_mb``, ``grad_reduce_dtype``,
  ``async_checkpoint`` (GPU default true: pinned snapshot + background write);
* ``trainer.extra.cuda_graph`` (single GPU, fused engine): after ``cuda_graph_warmup``
  eager steps the whole optimizer step is captured once as a hipGraph and replayed
  (:mod:`llmtrain.training.graph_step`) — for the launch-bound small presets;
* ``train/allreduce_ms`` (max over ranks) logs the exposed gradient all-reduce time of the flat
  reducer — the part of the communication NOT hidden behind the backward;
* non-finite gradients (the reference clips, steps and saves unconditionally,
  ``training/trainer.py:390-413``): a NaN/Inf global gradient norm skips the optimizer update
  (on device for the fused AdamW, no host sync), ``train/skipped_steps`` counts them at the log
  cadence (once one was skipped), ``trainer.extra.max_skipped_steps`` (default 8) consecutive skips seen at a log / save
  step raise, and a checkpoint is never written from non-finite weights or moments — the K8s
  auto-resume therefore never restarts from poisoned state.  ``trainer.extra.
  inject_nonfinite_grad_at_step`` (+ ``inject_nonfinite_rank``, default every rank) poisons that
  step's backward with NaN for fault-injection tests.
"""

from __future__ import annotations

import contextlib
import logging
import math
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Any

import torch
import torch.distributed as dist
from torch import nn

from llmtrain.config.schemas import RunConfig
from llmtrain.parallel.comm import last_probe
from llmtrain.parallel.ddp import unwrap, wrap_data_parallel
from llmtrain.parallel.dist import verify_replicas
from llmtrain.parallel.dist import DDPState
from llmtrain.registry import initialize_registries
from llmtrain.registry.data import get_data_module
from llmtrain.registry.models import get_model_adapter
from llmtrain.runtime.device import decorrelate_rank_streams, resolve_policy, seed_everything, settle_fused_path
from llmtrain.runtime.tuning import enable_tuned_gemms
from llmtrain.tracking import NullTracker, Tracker
from llmtrain.training.checkpoint import CheckpointManager, CheckpointPayload, restore_rng_states
from llmtrain.training.graph_step import GraphedStep, check_graphable
from llmtrain.training.optim import FusedAdamW, build_optimizer, fused_clip_coef

__all__ = ["TrainResult", "Trainer", "lr_lambda_factory"]

logger = logging.getLogger(__name__)


@dataclass(frozen=True)
class TrainResult:
    final_step: int
    final_loss: float
    final_val_loss: float | None
    total_time: float
    peak_memory: float
    val_metrics: dict[str, float] | None = None
    first_step_loss: float | None = None
    resumed_from_step: int | None = None
    parameter_count: int | None = None
    trainable_parameter_count: int | None = None


def lr_lambda_factory(warmup_steps: int, max_steps: int):  # type: ignore[no-untyped-def]
    """Linear warm-up 0→1 over ``warmup_steps``, then cosine 1→0 reaching 0 at ``max_steps``."""

    def lr_lambda(step: int) -> float:
        if step < warmup_steps:
            return step / warmup_steps
        if step >= max_steps:
            return 0.0
        if max_steps <= warmup_steps:
            return 1.0
        progress = (step - warmup_steps) / (max_steps - warmup_steps)
        return 0.5 * (1.0 + math.cos(math.pi * progress))

    return lr_lambda


def _drop_dense_mask(batch: dict[str, Any]) -> dict[str, Any]:
    """Drop an all-ones ``attention_mask`` while the batch is still on the host (a cheap CPU check,
    no device sync): without padding the masked mean IS the plain mean, and the fused engine /
    SDPA then take their unmasked kernels.  Malformed masks are kept so the adapter's validation
    still rejects them (reference ``models/gpt.py:221-252``)."""
    mask = batch.get("attention_mask")
    ids = batch.get("input_ids")
    if (
        torch.is_tensor(mask)
        and torch.is_tensor(ids)
        and mask.device.type == "cpu"
        and mask.dtype in (torch.bool, torch.long)
        and mask.shape == ids.shape
    ):
        if bool(mask.all()):
            return {k: v for k, v in batch.items() if k != "attention_mask"}
        if not bool(mask.any()):  # reference models/gpt.py:262-266, checked here without a device sync
            raise ValueError("attention_mask has no valid target tokens")
    return batch


def _to_device(batch: dict[str, Any], device: torch.device) -> dict[str, Any]:
    non_blocking = device.type == "cuda"
    batch = _drop_dense_mask(batch)
    return {
        k: v.to(device, non_blocking=non_blocking) if torch.is_tensor(v) else v for k, v in batch.items()
    }


def _loss_tensor(loss: torch.Tensor, metrics: dict[str, Any]) -> torch.Tensor:
    value = metrics.get("loss")
    tensor = getattr(value, "tensor", None)
    if isinstance(tensor, torch.Tensor):
        return tensor.detach().float()
    if value is not None and not isinstance(value, torch.Tensor):
        return torch.tensor(float(value), dtype=torch.float32, device=loss.device)
    return loss.detach().float()


class _Batches:
    """Endless iterator over a DataLoader that restarts it at each epoch boundary."""

    def __init__(self, loader: Any) -> None:
        self._loader = loader
        self._it = iter(loader)
        self.consumed = 0

    def next(self) -> dict[str, Any]:
        try:
            batch = next(self._it)
        except StopIteration:
            self._it = iter(self._loader)
            batch = next(self._it)
        self.consumed += 1
        return batch


class Trainer:
    def __init__(
        self,
        cfg: RunConfig,
        *,
        run_dir: Path | None = None,
        tracker: Tracker | None = None,
        ddp_state: DDPState | None = None,
    ) -> None:
        self._cfg = cfg
        self._tracker: Tracker = tracker or NullTracker()
        self._ddp_state = ddp_state
        initialize_registries()
        seed_everything(cfg.run.seed)

        self._adapter = get_model_adapter(cfg.model.name)()
        data_module = get_data_module(cfg.data.name)()
        model = self._adapter.build_model(cfg)
        tokenizer = self._adapter.build_tokenizer(cfg)
        data_module.setup(cfg, tokenizer=tokenizer)
        self._train_loader = data_module.train_dataloader()
        self._val_loader = data_module.val_dataloader()

        local_rank = ddp_state.local_rank if ddp_state is not None else 0
        supported = getattr(model, "fused_supported", None)
        fused_capable = hasattr(model, "prepare_runtime") and supported is not None
        policy = resolve_policy(cfg, local_rank=local_rank, fused_capable=fused_capable)
        if policy.use_fused and not supported(policy.device.type):
            # an error on GPU unless model.extra.allow_module_fallback (runtime/device.py)
            policy = settle_fused_path(policy, cfg, False)
            logger.warning("trainer: fused engine does not cover this model shape on %s; using the module path",
                           policy.device)
        self._policy = policy
        self._device = self._policy.device
        self.tuned_gemms = enable_tuned_gemms(self._device)  # shipped hipBLASLt solution table (GPU)
        model = model.to(self._device)
        if self._policy.use_fused:
            kw = {}
            if "residual_dtype" in cfg.model.extra:  # fused engine option (gpt_engine.RESIDUAL_MODES)
                kw["residual"] = str(cfg.model.extra["residual_dtype"])
            if "mlp_store" in cfg.model.extra:  # fused engine option: "u" | "gd"
                kw["mlp_store"] = str(cfg.model.extra["mlp_store"])
            engine = model.prepare_runtime(compute_dtype=self._policy.compute_dtype, **kw)
            engine.expect_deterministic = bool(cfg.run.deterministic)
        self._model: nn.Module = model
        if self._is_ddp_active:
            self._model = wrap_data_parallel(model, cfg, self._device)
            verify_replicas(model.parameters(), device=self._metric_device(), tag="after data-parallel wrap")
            decorrelate_rank_streams(self._rank)  # per-rank dropout masks; init stayed identical

        self._optimizer = build_optimizer(unwrap(self._model), cfg.trainer.lr, cfg.trainer.weight_decay)
        self._scheduler = self._build_scheduler(self._optimizer)
        self._ckpt_mgr: CheckpointManager | None = None
        if run_dir is not None:
            keep = int(cfg.trainer.extra.get("keep_last_k", 3))
            # on GPU the write goes to a background thread behind a pinned-memory snapshot
            # (trainer.extra.async_checkpoint, default on): the step pays the device-to-host copy only
            async_ckpt = self._device.type == "cuda" and bool(cfg.trainer.extra.get("async_checkpoint", True))
            self._ckpt_mgr = CheckpointManager(run_dir / "checkpoints", keep_last_k=keep, async_write=async_ckpt)
        self._run_dir = run_dir
        fail_at = cfg.trainer.extra.get("fail_at_step")
        if fail_at is not None and int(fail_at) <= cfg.trainer.save_every_steps:
            # the fault fires after the step's train_step and BEFORE its checkpoint: with no
            # checkpoint on disk a restarted job would start fresh and crash again every time
            raise ValueError(
                f"trainer.extra.fail_at_step={fail_at} must be greater than save_every_steps="
                f"{cfg.trainer.save_every_steps} (a restart must find a checkpoint to resume from)"
            )
        self.last_grad_norm: torch.Tensor | None = None
        self._skipped_host = [0, 0]  # module path: [total, consecutive] skipped steps
        self._max_skipped = int(cfg.trainer.extra.get("max_skipped_steps", 8))
        inject = cfg.trainer.extra.get("inject_nonfinite_grad_at_step")
        self._inject_at = None if inject is None else int(inject)
        self._current_step: int | None = None  # global step of the running train_step (fit only)
        self._graphed: GraphedStep | None = None
        if bool(cfg.trainer.extra.get("cuda_graph", False)):
            check_graphable(
                device=self._device, fused=self._policy.use_fused, optimizer=self._optimizer,
                ddp_active=self._is_ddp_active,
            )
            self._graphed = GraphedStep(
                device=self._device, optimizer=self._optimizer, eager=self._eager_step, body=self._captured_step,
                after=self._scheduler.step, warmup=int(cfg.trainer.extra.get("cuda_graph_warmup", 2)),
                engine=getattr(unwrap(self._model), "engine", None), dropout=float(cfg.model.dropout) > 0.0,
                run_seed=int(cfg.run.seed),
            )
        logger.info(
            "trainer: device=%s compute_dtype=%s fused=%s ddp=%s",
            self._device, self._policy.compute_dtype, self._policy.use_fused, self._is_ddp_active,
        )

    # -- properties ------------------------------------------------------------------------

    def _build_scheduler(self, optimizer: torch.optim.Optimizer) -> torch.optim.lr_scheduler.LambdaLR:
        fn = lr_lambda_factory(self._cfg.trainer.warmup_steps, self._cfg.trainer.max_steps)
        return torch.optim.lr_scheduler.LambdaLR(optimizer, lr_lambda=fn)

    @property
    def scheduler(self) -> torch.optim.lr_scheduler.LambdaLR:
        return self._scheduler

    @property
    def optimizer(self) -> torch.optim.Optimizer:
        return self._optimizer

    @property
    def model(self) -> nn.Module:
        return self._model

    @property
    def device(self) -> torch.device:
        return self._device

    @property
    def _is_main(self) -> bool:
        return self._ddp_state is None or self._ddp_state.is_main

    @property
    def _raw_model(self) -> nn.Module:
        return unwrap(self._model)

    @property
    def _rank(self) -> int:
        return self._ddp_state.rank if self._ddp_state is not None else 0

    @property
    def _world_size(self) -> int:
        return self._ddp_state.world_size if self._ddp_state is not None else 1

    @property
    def _is_ddp_active(self) -> bool:
        return self._ddp_state is not None and self._ddp_state.world_size > 1

    def _metric_device(self) -> torch.device:
        if dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl":
            return self._device
        return torch.device("cpu")

    # -- metric collectives (C4-C7) ------------------------------------------------------------

    def _reduce_metrics(self, **scalars: float) -> dict[str, float]:
        if not self._is_ddp_active:
            return dict(scalars)
        keys = list(scalars)
        t = torch.tensor([scalars[k] for k in keys], dtype=torch.float64, device=self._metric_device())
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return {k: float(v) for k, v in zip(keys, t.tolist())}

    def _gather_scalars(self, **scalars: float) -> list[dict[str, float]] | None:
        if not self._is_ddp_active:
            return [dict(scalars)]
        if not (dist.is_available() and dist.is_initialized()):
            return [dict(scalars)] if self._is_main else None
        keys = list(scalars)
        local = torch.tensor([scalars[k] for k in keys], dtype=torch.float64, device=self._metric_device())
        bucket = [torch.zeros_like(local) for _ in range(self._world_size)]
        dist.all_gather(bucket, local)
        if not self._is_main:
            return None
        return [{k: float(v) for k, v in zip(keys, t.tolist())} for t in bucket]

    # -- resume ------------------------------------------------------------------------------

    def restore(self, payload: CheckpointPayload) -> int:
        self._raw_model.load_state_dict(payload["model_state_dict"])
        self._optimizer.load_state_dict(payload["optimizer_state_dict"])
        self._scheduler.load_state_dict(payload["scheduler_state_dict"])
        restore_rng_states(payload["rng_states"])
        if self._is_ddp_active:
            ranks = (payload.get("llmtrain_extra") or {}).get("rank_rng_states")
            if isinstance(ranks, (list, tuple)) and len(ranks) == self._world_size:
                restore_rng_states(ranks[self._rank])  # this rank's own streams: exact continuation
            else:  # an older checkpoint or another world size: rank 0's streams, split again
                decorrelate_rank_streams(self._rank)
        store = getattr(self._raw_model, "flat_store", None)
        if store is not None:
            store.sync_shadow(force=True)
        step = int(payload["step"])
        logger.info("trainer: restored state from step %d", step)
        return step

    def _replay_batches(self, payload: CheckpointPayload, resumed_step: int) -> int:
        """Micro-batches this rank skips on resume so that no sample is trained twice or missed.

        Same world size as the checkpoint: exactly the batches each rank had consumed.  Another
        world size: the samplers shard one global order round-robin (``DistributedSampler``), so
        the checkpoint's ``batches_consumed × micro_batch × world`` samples are the prefix of that
        order already trained on; each new rank skips that many global samples' worth of its own
        batches (rounded down, with a warning naming the samples seen again).  A checkpoint
        without the record (reference / older files) falls back to ``step × grad_accum``."""
        accum = self._cfg.trainer.grad_accum_steps
        extra = payload.get("llmtrain_extra") or {}
        saved_world, consumed = extra.get("world_size"), extra.get("batches_consumed")
        if saved_world is None or consumed is None:
            if self._is_ddp_active:
                logger.warning("checkpoint: no world-size record; replaying step x grad_accum batches per rank")
            return resumed_step * accum
        saved_world, consumed = int(saved_world), int(consumed)
        if saved_world == self._world_size:
            return consumed
        saved_mb = int(payload["config"]["trainer"]["micro_batch_size"])
        seen = consumed * saved_mb * saved_world
        per_batch = self._cfg.trainer.micro_batch_size * self._world_size
        skip, again = divmod(seen, per_batch)
        logger.warning(
            "checkpoint: saved at world_size=%d, resuming at world_size=%d: continuing after global sample %d "
            "(%d batches per rank; %d samples of the interrupted position are trained again)",
            saved_world, self._world_size, seen, skip, again,
        )
        return skip

    def _gather_rng_states(self) -> list[Any] | None:
        """Every rank's RNG states (python / numpy / torch / HIP), gathered on the checkpoint
        cadence so rank 0's file can restore each rank's own dropout streams."""
        if not self._is_ddp_active:
            return None
        from llmtrain.training.checkpoint import capture_rng_states

        states: list[Any] = [None] * self._world_size
        dist.all_gather_object(states, capture_rng_states())
        return states

    def _resolve_resume_path(self, resume_from: str | Path) -> Path:
        candidate = Path(resume_from)
        if candidate.exists():
            if candidate.is_file():
                return candidate
            if candidate.is_dir():
                latest = CheckpointManager(candidate, keep_last_k=1).latest_checkpoint()
                if latest is None:
                    raise FileNotFoundError(f"No checkpoints found in {candidate}")
                return latest
            raise FileNotFoundError(f"Resume path {candidate} is not a file or directory")
        if candidate.suffix == ".pt":
            raise FileNotFoundError(f"Checkpoint file {candidate} does not exist")
        ckpt_dir = Path(self._cfg.output.root_dir) / str(resume_from) / "checkpoints"
        if not ckpt_dir.exists():
            raise FileNotFoundError(f"Checkpoint directory {ckpt_dir} does not exist")
        latest = CheckpointManager(ckpt_dir, keep_last_k=1).latest_checkpoint()
        if latest is None:
            raise FileNotFoundError(f"No checkpoints found in {ckpt_dir}")
        return latest

    # -- evaluation ----------------------------------------------------------------------------

    def _evaluate(self) -> tuple[dict[str, float], dict[str, float]] | None:
        if self._val_loader is None:
            return None
        was_training = self._model.training
        self._model.eval()
        loss_sum = torch.zeros((), dtype=torch.float64, device=self._device)
        tokens = 0
        with torch.no_grad(), self._policy.autocast():
            for batch in self._val_loader:
                batch = _to_device(batch, self._device)
                loss, metrics = self._adapter.compute_loss(self._raw_model, batch)
                n = batch["input_ids"].numel()
                loss_sum += _loss_tensor(loss, metrics).double() * n
                tokens += n
        if was_training:
            self._model.train()
        if tokens == 0:
            return {}, {}
        local_sum = float(loss_sum.item())
        local = {"val/loss": local_sum / tokens}
        if not self._is_ddp_active:
            return local, dict(local)
        red = self._reduce_metrics(loss_sum=local_sum, tok_count=float(tokens))
        glob = {"val/loss": red["loss_sum"] / red["tok_count"] if red["tok_count"] > 0 else 0.0}
        return local, glob

    # -- the loop ------------------------------------------------------------------------------

    def _sync_context(self, is_last_micro: bool) -> contextlib.AbstractContextManager[Any]:
        if not is_last_micro and hasattr(self._model, "no_sync"):
            return self._model.no_sync()
        return contextlib.nullcontext()

    def _optimizer_step(self) -> None:
        finish = getattr(self._model, "finish_gradient_sync", None)
        if finish is not None:
            finish()
        max_norm = self._cfg.trainer.max_grad_norm
        if isinstance(self._optimizer, FusedAdamW):
            # data parallel: the reducer summed each bucket's squared norm as its all-reduce finished
            bucket_sumsq = getattr(self._model, "grad_sumsq", None)
            sq = bucket_sumsq() if bucket_sumsq is not None else None
            norm, coef = fused_clip_coef(self._optimizer.store, max_norm, sumsq=sq)
            self._optimizer.step(grad_scale=coef)  # skips on device when coef is NaN
        else:
            norm = torch.nn.utils.clip_grad_norm_(self._model.parameters(), max_norm, error_if_nonfinite=False)
            if bool(torch.isfinite(norm)):  # module path: one host sync per step decides the skip
                self._optimizer.step()
                self._skipped_host[1] = 0
            else:
                self._skipped_host[0] += 1
                self._skipped_host[1] += 1
        self.last_grad_norm = norm  # pre-clip global L2 norm, device scalar (no host sync)
        self._scheduler.step()

    def skipped_steps(self) -> tuple[int, int]:
        """``(total, consecutive)`` optimizer steps skipped for a non-finite gradient norm (a host
        read of the fused optimizer's device counters: call it at a sync point)."""
        dev = getattr(self._optimizer, "skipped", None)
        if isinstance(dev, torch.Tensor):
            total, consecutive = (int(v) for v in dev.tolist())
            return total, consecutive
        return self._skipped_host[0], self._skipped_host[1]

    def _check_skips(self, step: int) -> int:
        """Raise once ``max_skipped_steps`` consecutive updates were skipped; returns the total."""
        total, consecutive = self.skipped_steps()
        if consecutive >= self._max_skipped:
            raise FloatingPointError(
                f"{consecutive} consecutive optimizer steps skipped for a non-finite gradient norm "
                f"(trainer.extra.max_skipped_steps={self._max_skipped}) at step {step}"
            )
        return total

    def _state_finite(self) -> bool:
        """Weights and optimizer moments all finite (checked before every checkpoint write)."""
        store = getattr(self._optimizer, "store", None)
        if store is not None:
            bufs = [store.master, self._optimizer.exp_avg, self._optimizer.exp_avg_sq]
        else:
            bufs = [p.detach() for p in self._raw_model.parameters()]
            for st in self._optimizer.state.values():
                bufs += [v for k, v in st.items() if k != "step" and isinstance(v, torch.Tensor)]
        flags = torch.stack([torch.isfinite(b).all() for b in bufs])
        return bool(flags.all())

    def _poison_factor(self) -> float:
        """Fault injection: NaN on the backward seed of the configured step (and rank), else 1."""
        if self._inject_at is None or self._current_step != self._inject_at:
            return 1.0
        target = self._cfg.trainer.extra.get("inject_nonfinite_rank")
        if target is not None and int(target) != self._rank:
            return 1.0
        return float("nan")

    def batch_stream(self) -> _Batches:
        """Endless iterator over this trainer's training DataLoader."""
        return _Batches(self._train_loader)

    def kernel_policy(self) -> contextlib.AbstractContextManager[Any]:
        """``run.deterministic`` for the HIP kernels (fixed-order reductions: bitwise-reproducible
        steps and resumes; false = the split-K / scatter atomics of the fast path), scoped to this
        trainer's own work: :meth:`fit` and :meth:`train_step` run under it, and the process-wide
        policy they found is restored when they return, so it never leaks into another trainer."""
        if self._device.type != "cuda":
            return contextlib.nullcontext()
        from llmtrain import ops

        return ops.kernel_policy(self._cfg.run.deterministic)

    def train_step(self, batches: _Batches) -> tuple[torch.Tensor, int]:
        """One optimizer step (all micro-batches, gradient sync, clip, AdamW, LR schedule).

        Returns the step's mean loss as a 0-d DEVICE tensor (no host sync) and its token count.
        ``bench.py`` times exactly this method.
        """
        with self.kernel_policy():
            return self._train_step(batches)

    def _train_step(self, batches: _Batches) -> tuple[torch.Tensor, int]:
        accum = self._cfg.trainer.grad_accum_steps
        if self._graphed is not None:  # trainer.extra.cuda_graph: replay the captured step
            host = [_drop_dense_mask(batches.next()) for _ in range(accum)]
            tokens = sum(int(b["input_ids"].numel()) for b in host)
            loss, self.last_grad_norm = self._graphed.step(host)
            return loss, tokens
        dev_batches = []
        tokens = 0
        for _ in range(accum):
            batch = _to_device(batches.next(), self._device)
            tokens += batch["input_ids"].numel()
            dev_batches.append(batch)
        loss, _ = self._eager_step(dev_batches)
        return loss, tokens

    def _eager_step(self, dev_batches: list[dict[str, Any]]) -> tuple[torch.Tensor, torch.Tensor]:
        """Micro-batch forward/backward (communication on the last only), clip, AdamW, LR step."""
        accum = len(dev_batches)
        self._optimizer.zero_grad()
        step_loss = torch.zeros((), dtype=torch.float32, device=self._device)
        poison = self._poison_factor()
        for micro, batch in enumerate(dev_batches):
            with self._sync_context(micro == accum - 1):
                with self._policy.autocast():
                    loss, metrics = self._adapter.compute_loss(self._model, batch)
                seed = loss / accum
                if poison != 1.0 and micro == accum - 1:
                    seed = seed * poison  # gradients only: the logged loss stays finite
                seed.backward()
            step_loss += _loss_tensor(loss, metrics)
        self._optimizer_step()
        assert self.last_grad_norm is not None
        return step_loss / accum, self.last_grad_norm

    def _captured_step(self, static: list[dict[str, Any]]) -> tuple[torch.Tensor, torch.Tensor]:
        """The body recorded into the hipGraph (single process, fused engine + fused AdamW): no
        host-side optimizer state changes here — :class:`GraphedStep` stages them per replay."""
        accum = len(static)
        self._optimizer.zero_grad()
        step_loss = torch.zeros((), dtype=torch.float32, device=self._device)
        for batch in static:
            with self._policy.autocast():
                loss, metrics = self._adapter.compute_loss(self._model, batch)
            (loss / accum).backward()
            step_loss += _loss_tensor(loss, metrics)
        norm, coef = fused_clip_coef(self._optimizer.store, self._cfg.trainer.max_grad_norm)
        self._optimizer.step_captured(grad_scale=coef)  # skips on device when coef is NaN
        return step_loss / accum, norm

    def _fault_rank(self) -> bool:
        """``trainer.extra.fail_rank`` (default: every rank) picks the rank that crashes."""
        target = self._cfg.trainer.extra.get("fail_rank")
        return target is None or int(target) == self._rank

    def _profiler(self) -> Any:
        spec = self._cfg.trainer.extra.get("profile")
        if not spec or self._run_dir is None or not self._is_main:
            return None
        from llmtrain.utils.profiling import StepProfiler

        return StepProfiler(spec, self._run_dir / "profile")

    def fit(
        self,
        *,
        max_steps_override: int | None = None,
        resume_from: str | Path | None = None,
    ) -> TrainResult:
        """Train to ``max_steps``; an asynchronous checkpoint still being written is flushed to disk
        before this returns or re-raises (a crash mid-run keeps the last complete checkpoint)."""
        try:
            with self.kernel_policy():
                result = self._fit(max_steps_override=max_steps_override, resume_from=resume_from)
        except BaseException:
            if self._ckpt_mgr is not None:
                try:
                    self._ckpt_mgr.wait()
                except Exception:  # the training error is the one to report
                    logger.exception("checkpoint: background write failed")
            raise
        if self._ckpt_mgr is not None:
            self._ckpt_mgr.wait()
        return result

    def _fit(self, *, max_steps_override: int | None, resume_from: str | Path | None) -> TrainResult:
        cfg = self._cfg.trainer
        self._model.train()
        max_steps = max_steps_override if max_steps_override is not None else cfg.max_steps
        accum = cfg.grad_accum_steps
        fail_at = self._cfg.trainer.extra.get("fail_at_step")
        if self._device.type == "cuda":
            torch.cuda.reset_peak_memory_stats(self._device)

        batches = _Batches(self._train_loader)
        start_step = 1
        resumed_from_step: int | None = None
        payload: Any = None
        if resume_from is not None:
            path = self._resolve_resume_path(resume_from)
            payload = CheckpointManager(path.parent, keep_last_k=1).load(path)
            if payload["config"] != self._cfg.model_dump():
                logger.warning("checkpoint: config mismatch detected; using current config for resume")
            resumed_from_step = self.restore(payload)
            if self._is_ddp_active:
                verify_replicas(self._raw_model.parameters(), device=self._metric_device(), tag="after resume")
            start_step = resumed_from_step + 1
            if start_step > max_steps:
                logger.info(
                    "trainer: resume step %d >= max_steps %d; no further steps", resumed_from_step, max_steps
                )
        if self._is_main:
            self._tracker.log_params(self._cfg.model_dump())
            probe = last_probe() if self._is_ddp_active else None
            if probe is not None:  # the startup all-reduce probe of setup_ddp (parallel/comm.py)
                self._tracker.log_metrics({"ddp/allreduce_busbw_gbps": probe.busbw_gbps}, step=0)
        n_params = sum(p.numel() for p in self._raw_model.parameters())
        n_trainable = sum(p.numel() for p in self._raw_model.parameters() if p.requires_grad)

        t_start = time.perf_counter()
        if resumed_from_step:
            # Replay the data order: each rank skips its own shard's batches (deterministic
            # samplers), which keeps ranks aligned — the reference skips only without DDP.
            for _ in range(self._replay_batches(payload, resumed_from_step)):
                batches.next()

        first_step_loss: float | None = None
        final_val_loss: float | None = None
        final_val_metrics: dict[str, float] | None = None
        step_loss = 0.0
        tokens_local_total = 0
        tokens_global_total = 0
        interval_loss = torch.zeros((), dtype=torch.float32, device=self._device)
        interval_steps = 0
        interval_tokens = 0
        interval_t0 = time.perf_counter()
        last_step_loss_dev: torch.Tensor | None = None
        profiler = self._profiler()

        for step in range(start_step, max_steps + 1):
            if profiler is not None:
                profiler.before_step(step)
            self._current_step = step
            step_loss_dev, step_tokens = self.train_step(batches)
            self._current_step = None
            if fail_at is not None and step == int(fail_at) and resumed_from_step is None and self._fault_rank():
                # simulated crash of one incarnation of the job: a resumed run does not re-fire it
                raise RuntimeError(f"fault injection: trainer.extra.fail_at_step={fail_at} (rank {self._rank})")
            last_step_loss_dev = step_loss_dev
            tokens_local_total += step_tokens
            if step == 1:
                first_step_loss = float(step_loss_dev.item())

            if step % cfg.save_every_steps == 0 or step == max_steps:
                self._check_skips(step)
                rank_rng = self._gather_rng_states()  # a collective: every rank, every save step
                if self._ckpt_mgr is not None and self._is_main:
                    if not self._state_finite():
                        raise FloatingPointError(
                            f"refusing to checkpoint step {step}: non-finite weights or optimizer moments"
                        )
                    extra = {"world_size": self._world_size, "batches_consumed": batches.consumed}
                    if rank_rng is not None:
                        extra["rank_rng_states"] = rank_rng
                    self._ckpt_mgr.save(step, self._raw_model, self._optimizer, self._scheduler, self._cfg, extra=extra)

            interval_loss += step_loss_dev
            interval_steps += 1
            interval_tokens += step_tokens

            if step % cfg.log_every_steps == 0 or step == max_steps:
                avg_loss = float(interval_loss.item()) / interval_steps  # the interval's one sync
                interval_time = time.perf_counter() - interval_t0
                step_time = interval_time / interval_steps
                tps = interval_tokens / interval_time if interval_time > 0 else 0.0
                lr = float(self._scheduler.get_last_lr()[0])
                if not math.isfinite(avg_loss) and self._cfg.trainer.extra.get("halt_on_nan", True):
                    raise FloatingPointError(f"non-finite training loss {avg_loss} at step {step}")
                # logged once a step was skipped (the reference's metric set stays exact otherwise)
                skipped_total = self._check_skips(step)
                skip_metric = {"train/skipped_steps": float(skipped_total)} if skipped_total else {}
                extra_metrics = {**skip_metric, **self._device_metrics(tps)}
                if self._is_ddp_active:
                    comm_ms = self._exposed_comm_ms()
                    per_rank = self._gather_scalars(
                        avg_loss=avg_loss, lr=lr, tokens_per_sec=tps, step_time=step_time,
                        tokens_total=float(tokens_local_total), allreduce_ms=comm_ms,
                    )
                    worst_comm_ms = comm_ms
                    if per_rank is not None:
                        worst_comm_ms = max(v["allreduce_ms"] for v in per_rank)
                        for r, vals in enumerate(per_rank):
                            self._tracker.log_metrics(
                                {
                                    f"train/loss_rank_{r}": vals["avg_loss"],
                                    f"train/lr_rank_{r}": vals["lr"],
                                    f"train/tokens_per_sec_rank_{r}": vals["tokens_per_sec"],
                                    f"train/step_time_sec_rank_{r}": vals["step_time"],
                                    f"train/tokens_total_rank_{r}": vals["tokens_total"],
                                    f"train/allreduce_ms_rank_{r}": vals["allreduce_ms"],
                                },
                                step=step,
                            )
                    red = self._reduce_metrics(
                        loss_sum=float(interval_loss.item()), steps=float(interval_steps), tokens=float(interval_tokens)
                    )
                    if self._is_main:
                        tokens_global_total += int(red["tokens"])
                        global_tps = red["tokens"] / interval_time if interval_time > 0 else 0.0
                        self._tracker.log_metrics(
                            {
                                "train/loss": red["loss_sum"] / red["steps"],
                                "train/lr": lr,
                                "train/tokens_per_sec": global_tps,
                                "train/tokens_total": float(tokens_global_total),
                                "train/step_time_sec": step_time,
                                "train/allreduce_ms": worst_comm_ms,
                                **skip_metric,
                                **self._device_metrics(global_tps / self._world_size),
                            },
                            step=step,
                        )
                elif self._is_main:
                    self._tracker.log_metrics(
                        {
                            "train/loss": avg_loss,
                            "train/lr": lr,
                            "train/tokens_per_sec": tps,
                            "train/step_time_sec": step_time,
                            "train/tokens_total": float(tokens_local_total),
                            **extra_metrics,
                        },
                        step=step,
                    )
                logger.info(
                    "step=%d/%d  loss=%.4f  lr=%.6e  tokens_per_sec=%.1f  step_time=%.4fs",
                    step, max_steps, avg_loss, lr, tps, step_time,
                )
                interval_loss.zero_()
                interval_steps = 0
                interval_tokens = 0
                interval_t0 = time.perf_counter()

            if step % cfg.eval_every_steps == 0 or step == max_steps:
                result = self._evaluate()
                if result is not None:
                    local_val, global_val = result
                    if self._is_ddp_active:
                        per_rank = self._gather_scalars(val_loss=local_val.get("val/loss", 0.0))
                        if per_rank is not None:
                            for r, vals in enumerate(per_rank):
                                self._tracker.log_metrics({f"val/loss_rank_{r}": vals["val_loss"]}, step=step)
                    if self._is_main:
                        self._tracker.log_metrics(global_val, step=step)
                    effective = global_val if self._is_main else local_val
                    if effective:
                        final_val_metrics = effective
                        if "val/loss" in effective:
                            final_val_loss = effective["val/loss"]
                        text = "  ".join(f"{k}={v:.4f}" for k, v in sorted(effective.items()))
                        logger.info("val_step=%d/%d  %s", step, max_steps, text)
                interval_t0 = time.perf_counter() if interval_steps == 0 else interval_t0
            if profiler is not None:
                profiler.after_step(step)

        if last_step_loss_dev is not None:
            step_loss = float(last_step_loss_dev.item())
        if profiler is not None:
            profiler.close()
        total_time = time.perf_counter() - t_start
        peak = 0.0
        if self._device.type == "cuda":
            peak = torch.cuda.max_memory_allocated(self._device) / 2**30
        return TrainResult(
            final_step=max_steps,
            final_loss=step_loss,
            final_val_loss=final_val_loss,
            total_time=total_time,
            peak_memory=peak,
            val_metrics=final_val_metrics,
            first_step_loss=first_step_loss,
            resumed_from_step=resumed_from_step,
            parameter_count=n_params,
            trainable_parameter_count=n_trainable,
        )

    def _exposed_comm_ms(self) -> float:
        """Exposed gradient all-reduce time of the last step (ms): the flat reducer's wait after
        the backward's last kernel.  torch DDP (module path) does not expose it: 0.0 there."""
        probe = getattr(self._model, "exposed_comm_ms", None)
        value = probe() if probe is not None else None
        return float(value) if value is not None else 0.0

    def _device_metrics(self, tokens_per_sec_per_gpu: float) -> dict[str, float]:
        """GPU-only extras: model FLOPs utilisation (vs dense bf16 peak) and peak memory."""
        if self._device.type != "cuda":
            return {}
        from llmtrain.utils.flops import mfu, training_flops_per_token

        per_tok = training_flops_per_token(self._raw_model, self._cfg.model.block_size)
        return {
            "train/mfu": mfu(tokens_per_sec_per_gpu, per_tok),
            "train/peak_mem_gb": torch.cuda.max_memory_allocated(self._device) / 2**30,
        }
