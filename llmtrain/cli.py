"""``llmtrain`` command line (reference ``cli.py:102-344``).

``llmtrain [-v] [--version] {train,validate,print-config} --config PATH [--run-id ID]
[--dry-run] [--json] [--resume RUN_ID|DIR|FILE]``

``llmtrain generate --config PATH [--checkpoint RUN_ID|DIR|FILE] --prompt TEXT ...`` samples
from a trained ``gpt`` checkpoint with the KV-cached sampler of :mod:`llmtrain.inference` (the
reference has this only as notebook code, notebooks/trained_vs_random_completion.ipynb).

Exit codes: 0 success, 2 config/registry error, 1 training or dry-run failure.  Only rank 0
creates the run directory, writes ``config.yaml``/``meta.json``, owns a real tracker and prints
the summary.  In ``--json`` mode every logger used during the run writes to stderr so stdout
carries exactly one JSON document.
"""

from __future__ import annotations

import argparse
import io
import json
import logging
import os
import sys
from collections.abc import Callable, Iterator, Sequence
from contextlib import contextmanager
from pathlib import Path
from typing import Any, TextIO

import yaml

from llmtrain import __version__
from llmtrain.config.loader import ConfigLoadError, load_and_validate_config
from llmtrain.config.schemas import LoggingConfig, RunConfig
from llmtrain.parallel.dist import DDPState, setup_ddp, teardown_ddp
from llmtrain.registry import initialize_registries
from llmtrain.registry.core import RegistryError
from llmtrain.registry.data import get_data_module
from llmtrain.registry.models import get_model_adapter
from llmtrain.tracking import MLflowTracker, NullTracker, Tracker
from llmtrain.training import Trainer
from llmtrain.training.dry_run import run_dry_run
from llmtrain.utils.logging import configure_logging
from llmtrain.utils.metadata import generate_meta, write_meta_json
from llmtrain.utils.run_dir import create_run_directory, write_resolved_config
from llmtrain.utils.run_id import generate_run_id
from llmtrain.utils.summary import format_run_summary

__all__ = ["build_parser", "main"]

_LEVELS = {name: getattr(logging, name) for name in ("DEBUG", "INFO", "WARNING", "ERROR")}


def _configure_logger(
    config_logging: LoggingConfig,
    *,
    verbose: int,
    log_dir: Path | None = None,
    stream: TextIO | None = None,
) -> logging.Logger:
    level = logging.DEBUG if verbose > 0 else _LEVELS.get(config_logging.level, logging.INFO)
    file_name = config_logging.file_name
    if log_dir is not None:
        file_name = str(log_dir / file_name)
    return configure_logging(
        level=level,
        json_output=config_logging.json_output,
        log_to_file=config_logging.log_to_file,
        file_name=file_name,
        stream=stream,
    )


def _emit_config_error(error: ConfigLoadError, *, json_output: bool) -> None:
    if json_output:
        body = {"status": "error", "message": error.message, "details": error.details, "errors": error.errors}
        print(json.dumps(body, indent=2, default=str), file=sys.stderr)
        return
    print(f"Config error: {error.message}", file=sys.stderr)
    if error.details:
        print(error.details, file=sys.stderr)


def _create_tracker(config: RunConfig, logger: logging.Logger) -> Tracker:
    ml = config.mlflow
    if not ml.enabled:
        return NullTracker()
    try:
        return MLflowTracker(tracking_uri=ml.tracking_uri, experiment=ml.experiment, run_name=ml.run_name)
    except RuntimeError as exc:
        logger.warning("MLflow unavailable; falling back to NullTracker: %s", exc)
        return NullTracker()


def _log_run_artifacts(tracker: Tracker, run_dir: Path) -> None:
    for name in ("config.yaml", "meta.json"):
        path = run_dir / name
        if path.exists():
            tracker.log_artifact(path, artifact_path="artifacts")


class _StderrHandler(logging.StreamHandler):
    """Writes to whatever ``sys.stderr`` is at emit time (robust to stream swaps in embedders)."""

    def __init__(self) -> None:
        super().__init__(sys.stderr)

    @property  # type: ignore[override]
    def stream(self) -> TextIO:
        return sys.stderr

    @stream.setter
    def stream(self, value: TextIO) -> None:
        pass


def _route_to_stderr(name: str, template: logging.Logger) -> logging.Logger:
    """Send a child logger's records to stderr only (``--json`` keeps stdout clean)."""
    child = logging.getLogger(name)
    child.setLevel(template.level)
    child.handlers.clear()
    handler = _StderrHandler()
    handler.setFormatter(template.handlers[0].formatter if template.handlers else None)
    child.addHandler(handler)
    child.propagate = False
    return child


@contextmanager
def _stdout_reserved(enabled: bool) -> Iterator[Callable[[str], None]]:
    """In ``--json`` mode give the run's fd 1 to stderr and yield a writer for the real stdout.

    Native libraries write to fd 1 behind Python's back — under ``torchrun`` libgloo prints
    ``[Gloo] Rank r is connected to ...`` from every rank, RCCL may print its banner — so routing
    the loggers to stderr is not enough to keep stdout one JSON document (reference contract:
    cli.py:281-288, 315-322; tests/test_distributed.py:733-761).  fd 1 is pointed at fd 2 before
    the process group exists and restored afterwards; only the summary goes to the saved fd."""
    if not enabled:
        yield lambda text: print(text)
        return
    sys.stdout.flush()
    try:
        fd = sys.stdout.fileno()
    except (AttributeError, OSError, io.UnsupportedOperation):
        # stdout is a Python object (in-process capture): no native writer can reach it
        yield lambda text: print(text)
        return
    saved = os.dup(fd)
    os.dup2(sys.stderr.fileno(), fd)

    def write(text: str) -> None:
        data = (text + "\n").encode()
        while data:
            data = data[os.write(saved, data):]

    try:
        yield write
    finally:
        sys.stdout.flush()
        os.dup2(saved, fd)
        os.close(saved)


def build_parser() -> argparse.ArgumentParser:
    parser = argparse.ArgumentParser(
        prog="llmtrain",
        description="MI355X-native GPT training: validate configs, inspect them, and run training.",
    )
    parser.add_argument("--version", action="version", version=f"%(prog)s {__version__}")
    parser.add_argument("-v", "--verbose", action="count", default=0, help="Increase log verbosity.")
    common = argparse.ArgumentParser(add_help=False)
    common.add_argument("--config", required=True, help="Path to the YAML configuration file.")
    common.add_argument("--run-id", help="Override the run ID.")
    common.add_argument("--dry-run", action="store_true", help="Forward-only sanity run, no training.")
    common.add_argument("--json", action="store_true", help="Emit machine-readable JSON output.")
    sub = parser.add_subparsers(dest="command", required=True)
    train = sub.add_parser("train", parents=[common], help="Run (or dry-run) training.")
    train.add_argument("--resume", default=None, help="Resume from a run_id, checkpoint dir or .pt file.")
    sub.add_parser("validate", parents=[common], help="Validate a config file.")
    sub.add_parser("print-config", parents=[common], help="Print the resolved config with defaults.")
    gen = sub.add_parser("generate", help="Sample text from a trained gpt checkpoint (KV-cached).")
    gen.add_argument("--config", required=True, help="Path to the YAML configuration file.")
    gen.add_argument("--json", action="store_true", help="Emit machine-readable JSON output.")
    gen.add_argument("--checkpoint", default=None,
                     help="run_id, run/checkpoints dir or step_*.pt (omit: random-init weights).")
    gen.add_argument("--prompt", action="append", required=True, help="Prompt text (repeatable).")
    gen.add_argument("--max-new-tokens", type=int, default=48)
    gen.add_argument("--temperature", type=float, default=0.8, help="<= 0 means greedy argmax.")
    gen.add_argument("--top-k", type=int, default=40, help="0 disables the top-k cutoff.")
    gen.add_argument("--seed", type=int, default=1234)
    gen.add_argument("--top-next", type=int, default=0, help="Also list the k most likely next tokens.")
    gen.add_argument("--device", default=None, help="Override run.device (cpu | cuda).")
    gen.add_argument("--no-cache", action="store_true", help="Recompute the full context every step.")
    gen.add_argument("--graph", action="store_true",
                     help="Decode through a captured hipGraph (one graph launch per token on GPU).")
    return parser


def _load(args: argparse.Namespace) -> RunConfig | None:
    try:
        config, _, _ = load_and_validate_config(args.config)
    except ConfigLoadError as exc:
        _emit_config_error(exc, json_output=args.json)
        return None
    _configure_logger(config.logging, verbose=args.verbose, stream=sys.stderr if args.json else None)
    return config


def _handle_validate(args: argparse.Namespace) -> int:
    if _load(args) is None:
        return 2
    print(json.dumps({"status": "ok"}, indent=2) if args.json else "Config validation succeeded.")
    return 0


def _handle_print_config(args: argparse.Namespace) -> int:
    config = _load(args)
    if config is None:
        return 2
    payload = config.model_dump()
    if args.json:
        print(json.dumps(payload, indent=2))
    else:
        print(yaml.safe_dump(payload, sort_keys=False), end="")
    return 0


def _handle_train(args: argparse.Namespace) -> int:
    try:
        config, raw_path, resolved_path = load_and_validate_config(args.config)
    except ConfigLoadError as exc:
        _emit_config_error(exc, json_output=args.json)
        return 2
    with _stdout_reserved(bool(args.json)) as emit:
        return _train(args, config, raw_path, resolved_path, emit)


def _train(
    args: argparse.Namespace, config: RunConfig, raw_path: str, resolved_path: Any, emit: Callable[[str], None]
) -> int:
    ddp_state: DDPState | None = setup_ddp(config) if config.ddp.enabled else None
    is_main = ddp_state is None or ddp_state.is_main
    root = config.output.root_dir
    run_id = args.run_id or config.output.run_id or generate_run_id(config.run.name, root)
    run_dir = create_run_directory(root, run_id) if is_main else Path(root) / run_id
    # Non-main ranks log to stdout only (the reference wrote ./train.log in the CWD, Q10).
    log_cfg = config.logging if is_main else config.logging.model_copy(update={"log_to_file": False})
    logger = _configure_logger(
        log_cfg,
        verbose=args.verbose,
        log_dir=run_dir / "logs" if is_main else None,
        stream=sys.stderr if args.json else None,
    )
    if is_main:
        if config.output.save_config_copy:
            write_resolved_config(run_dir, config)
        if config.output.save_meta_json:
            meta = generate_meta(
                run_id=run_id, run_name=config.run.name, config_path=raw_path,
                resolved_config_path=str(resolved_path),
            )
            write_meta_json(run_dir, meta)

    initialize_registries()
    try:
        get_model_adapter(config.model.name)
        get_data_module(config.data.name)
    except RegistryError as exc:
        _emit_config_error(ConfigLoadError(str(exc)), json_output=args.json)
        if ddp_state is not None:
            teardown_ddp()
        return 2

    tracker: Tracker = _create_tracker(config, logger) if is_main else NullTracker()
    try:
        tracker.start_run(run_name=config.mlflow.run_name or run_id)
        summary: Any
        if args.dry_run:
            dry_logger = _route_to_stderr("llmtrain.dry_run", logger) if args.json else logger
            try:
                dry = run_dry_run(config, logger=dry_logger)
            except Exception as exc:
                print(f"Dry-run failed: {exc}", file=sys.stderr)
                return 1
            summary = format_run_summary(
                config=config, run_id=run_id, run_dir=run_dir, json_output=args.json,
                resolved_model_adapter=dry.resolved_model_adapter,
                resolved_data_module=dry.resolved_data_module,
                dry_run_steps_executed=dry.steps_executed,
            )
        else:
            if args.json:
                _route_to_stderr("llmtrain.training.trainer", logger)
            resume_from = getattr(args, "resume", None)
            if resume_from is not None:
                logger.info("Resuming from: %s", resume_from)
            try:
                trainer = Trainer(
                    config, run_dir=run_dir if is_main else None, tracker=tracker, ddp_state=ddp_state
                )
                result = trainer.fit(resume_from=resume_from)
            except Exception as exc:
                logger.debug("training failed", exc_info=True)
                print(f"Training failed: {exc}", file=sys.stderr)
                return 1
            summary = format_run_summary(
                config=config, run_id=run_id, run_dir=run_dir, json_output=args.json,
                train_result=result, resumed_from=resume_from,
            )
        if is_main:
            _log_run_artifacts(tracker, run_dir)
            emit(json.dumps(summary, indent=2) if args.json else summary)
    finally:
        tracker.end_run()
        if ddp_state is not None:
            teardown_ddp()
    return 0


def _resolve_checkpoint(spec: str, root_dir: str) -> Path:
    """A ``.pt`` file, a directory holding ``step_*.pt`` (or its run dir), or a run_id under
    ``output.root_dir`` — the same forms ``train --resume`` accepts."""
    from llmtrain.training.checkpoint import CheckpointManager

    path = Path(spec)
    if path.is_file():
        return path
    candidates = [path, path / "checkpoints"] if path.is_dir() else [Path(root_dir) / spec / "checkpoints"]
    for cand in candidates:
        if cand.is_dir():
            latest = CheckpointManager(cand).latest_checkpoint()
            if latest is not None:
                return latest
    raise FileNotFoundError(f"no checkpoint found for {spec!r}")


def _handle_generate(args: argparse.Namespace) -> int:
    args.verbose = getattr(args, "verbose", 0)
    config = _load(args)
    if config is None:
        return 2
    import torch

    from llmtrain.inference import generate_text, top_next_tokens
    from llmtrain.models.gpt import GPT
    from llmtrain.runtime.device import seed_everything
    from llmtrain.training.checkpoint import CheckpointManager

    initialize_registries()
    try:
        adapter = get_model_adapter(config.model.name)()
    except RegistryError as exc:
        print(f"Registry error: {exc}", file=sys.stderr)
        return 2
    try:
        seed_everything(config.run.seed)
        model = adapter.build_model(config)
        if not isinstance(model, GPT):
            print(f"generate supports the causal 'gpt' model, not {config.model.name!r}", file=sys.stderr)
            return 2
        tokenizer = adapter.build_tokenizer(config)
        source = "random-init"
        if args.checkpoint:
            ckpt = _resolve_checkpoint(args.checkpoint, config.output.root_dir)
            payload = CheckpointManager(ckpt.parent).load(ckpt)
            model.load_state_dict(payload["model_state_dict"])
            source = str(ckpt)
        want = args.device or config.run.device
        device = torch.device("cuda" if want in ("cuda", "rocm") and torch.cuda.is_available() else "cpu")
        model = model.to(device).eval()
        results: list[dict[str, Any]] = []
        for prompt in args.prompt:
            ids = tokenizer.encode(prompt)
            if not ids or max(ids) >= model.vocab_size:
                raise ValueError(f"prompt {prompt!r} encodes to no tokens or to ids >= vocab_size {model.vocab_size}")
            text = generate_text(
                model, tokenizer, prompt, max_new_tokens=args.max_new_tokens, temperature=args.temperature,
                top_k=args.top_k if args.top_k > 0 else None, seed=args.seed, use_cache=not args.no_cache,
                use_graph=args.graph,
            )
            entry: dict[str, Any] = {"prompt": prompt, "completion": text}
            if args.top_next > 0:
                entry["top_next"] = [[tok, p] for tok, p in top_next_tokens(model, tokenizer, prompt, k=args.top_next)]
            results.append(entry)
    except Exception as exc:  # noqa: BLE001 - CLI boundary: report and exit 1
        print(f"Generation failed: {exc}", file=sys.stderr)
        return 1
    if args.json:
        print(json.dumps({"checkpoint": source, "device": str(device), "results": results}, indent=2))
    else:
        for entry in results:
            print(f"=== prompt ===\n{entry['prompt']}\n=== completion ({source}) ===\n{entry['completion']}")
            for tok, p in entry.get("top_next", []):
                print(f"{tok!r}: {p:.4f}")
    return 0


def main(argv: Sequence[str] | None = None) -> int:
    args = build_parser().parse_args(argv)
    handlers = {
        "validate": _handle_validate,
        "print-config": _handle_print_config,
        "train": _handle_train,
        "generate": _handle_generate,
    }
    handler = handlers.get(args.command)
    if handler is None:
        print(f"Unknown command: {args.command}", file=sys.stderr)
        return 1
    return handler(args)
