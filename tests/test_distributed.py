"""Data-parallel runtime (reference tests/test_distributed.py), exercised with REAL multi-process
gloo groups on CPU (world_size 2): rank/env resolution, the flat-buffer bucketed reducer of the
fused engine (gradients == mean of the per-rank gradients, no_sync accumulation), the Trainer's
DDP metric naming / rank-0-only I/O, and a torchrun end-to-end run of the CLI."""

from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from llmtrain.config.schemas import RunConfig
from llmtrain.parallel.dist import DDPState, resolve_backend, setup_ddp, teardown_ddp
from llmtrain.parallel.reducer import plan_buckets
from llmtrain.runtime.flat import Segment

from conftest import REPO, minimal_payload


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(autouse=True)
def _teardown():
    yield
    if dist.is_initialized():
        dist.destroy_process_group()


def test_ddp_state_invariant() -> None:
    DDPState(rank=0, world_size=2, local_rank=0, is_main=True)
    with pytest.raises(ValueError):
        DDPState(rank=1, world_size=2, local_rank=1, is_main=True)


def test_setup_single_rank_from_env_and_idempotent(monkeypatch: pytest.MonkeyPatch) -> None:
    for k, v in {"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                 "MASTER_PORT": str(_free_port())}.items():
        monkeypatch.setenv(k, v)
    cfg = RunConfig.model_validate(minimal_payload(ddp={"enabled": True}))
    state = setup_ddp(cfg)
    assert state == DDPState(0, 1, 0, True) and dist.get_backend() == "gloo"
    assert setup_ddp(cfg) == state  # already initialised: returns the existing state
    teardown_ddp()
    assert not dist.is_initialized()


def test_config_fallback_and_errors(monkeypatch: pytest.MonkeyPatch) -> None:
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.delenv("MASTER_PORT", raising=False)
    port = _free_port()
    cfg = RunConfig.model_validate(minimal_payload(ddp={"enabled": True, "rank": 0, "world_size": 1, "local_rank": 0,
                                                        "master_addr": "127.0.0.1", "master_port": port}))
    assert setup_ddp(cfg).world_size == 1 and os.environ["MASTER_PORT"] == str(port)
    teardown_ddp()
    missing = RunConfig.model_validate(minimal_payload(ddp={"enabled": True}))
    with pytest.raises(RuntimeError, match="not found in env"):
        setup_ddp(missing)
    monkeypatch.setenv("RANK", "zero")
    with pytest.raises(RuntimeError, match="must be an integer"):
        setup_ddp(missing)


def test_backend_aliases() -> None:
    for name, want in (("gloo", "gloo"), ("nccl", "nccl"), ("rccl", "nccl")):
        cfg = RunConfig.model_validate(minimal_payload(ddp={"backend": name}))
        assert resolve_backend(cfg) == want


def test_plan_buckets_contiguous_and_capped() -> None:
    segs = [Segment("a", 0, 10), Segment("b", 10, 30), Segment("c", 40, 5), Segment("d", 45, 100)]
    buckets = plan_buckets(segs, cap_bytes=120)
    assert [b.segments for b in buckets] == [("a", "b"), ("c", "d")]
    assert buckets[1].start == 40 and buckets[1].numel == 105


# ----------------------------------------------------------------------------------------------
# real 2-process gloo worlds


def _init(rank: int, world: int, port: int) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)


def _reducer_worker(rank: int, world: int, port: int, out_dir: str) -> None:
    _init(rank, world, port)
    from llmtrain.models.gpt import GPT
    from llmtrain.parallel.reducer import FlatDataParallel

    torch.manual_seed(1234 + rank)  # different init per rank: the wrapper must broadcast rank 0's
    model = GPT(vocab_size=50, block_size=8, d_model=64, n_layers=2, n_heads=2, d_ff=64, dropout=0.0)
    model.prepare_runtime(compute_dtype=torch.float32)
    ddp = FlatDataParallel(model, bucket_cap_mb=0.01)
    assert len(ddp.buckets) > 2
    from llmtrain.parallel.dist import ReplicaMismatchError, verify_replicas

    verify_replicas(model.parameters(), device=torch.device("cpu"), tag="test")  # broadcast made them equal
    if rank == 1:
        with torch.no_grad():
            model.flat_store.master[0] += 1.0  # diverge one rank ...
    try:
        verify_replicas(model.parameters(), device=torch.device("cpu"), tag="diverged")
        raise AssertionError("mismatch not detected")
    except ReplicaMismatchError:
        pass  # ... and every rank sees it
    if rank == 1:
        with torch.no_grad():
            model.flat_store.master[0] -= 1.0
    verify_replicas(model.parameters(), device=torch.device("cpu"), tag="restored")
    g = torch.Generator().manual_seed(99 + rank)
    batches = [torch.randint(0, 50, (2, 8), generator=g) for _ in range(2)]
    model.flat_store.zero_grad()
    with ddp.no_sync():
        (ddp.fused_loss(batches[0], batches[0]) / 2).backward()
    (ddp.fused_loss(batches[1], batches[1]) / 2).backward()
    ddp.finish_gradient_sync()
    # bucket-wise squared norms (summed as each bucket's reduction finished) == one pass over the
    # reduced flat gradient, which is what fused_clip_coef computes without a reducer
    from llmtrain.training.optim import fused_clip_coef

    sq = ddp.grad_sumsq()
    assert sq is not None
    norm_b, coef_b = fused_clip_coef(model.flat_store, 0.5, sumsq=sq)
    norm_g, coef_g = fused_clip_coef(model.flat_store, 0.5)
    torch.testing.assert_close(norm_b, norm_g, rtol=1e-6, atol=0.0)
    torch.testing.assert_close(coef_b, coef_g, rtol=1e-6, atol=0.0)
    torch.save(
        {"params": model.flat_store.master.clone(), "grad": model.flat_store.grad.clone(), "batches": batches},
        Path(out_dir) / f"rank{rank}.pt",
    )
    with ddp.no_sync():  # an accumulation micro-step has no synchronised gradients yet
        ddp.fused_loss(batches[0], batches[0]).backward()
    assert ddp.grad_sumsq() is not None  # still the last synchronised step's until the next arm
    ddp.fused_loss(batches[0], batches[0])  # arms the next synchronised step ...
    assert ddp.grad_sumsq() is None  # ... whose norm is not known before its backward
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_flat_reducer_averages_gradients(tmp_path: Path, world: int) -> None:
    """The flat bucketed reducer at 2 and 4 gloo ranks (the 8-GPU path's logic beyond one pair):
    rank 0's parameters broadcast at wrap time, every rank ends with the average of all ranks'
    gradients, and the bucket-wise norm equals the global one."""
    mp.spawn(_reducer_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    ranks = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    r0 = ranks[0]
    for other in ranks[1:]:
        assert torch.equal(r0["params"], other["params"])  # broadcast at wrap time
        assert torch.allclose(r0["grad"], other["grad"])
    # reference: per-rank gradients computed independently, then averaged
    from llmtrain.models.gpt import GPT

    grads = []
    for rank_data in ranks:
        model = GPT(vocab_size=50, block_size=8, d_model=64, n_layers=2, n_heads=2, d_ff=64, dropout=0.0)
        model.prepare_runtime(compute_dtype=torch.float32)
        with torch.no_grad():
            model.flat_store.master.copy_(r0["params"])
        model.flat_store.sync_shadow(force=True)
        model.flat_store.zero_grad()
        for b in rank_data["batches"]:
            (model.fused_loss(b, b) / 2).backward()
        grads.append(model.flat_store.grad.clone())
    torch.testing.assert_close(r0["grad"], sum(grads) / world, atol=1e-6, rtol=1e-5)


def _trainer_worker(rank: int, world: int, port: int, out_dir: str, fused: bool) -> None:
    _init(rank, world, port)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from llmtrain.training.trainer import Trainer

    class Recorder:
        def __init__(self) -> None:
            self.metrics: list[tuple[int, dict]] = []

        def start_run(self, *a, **k): ...
        def log_params(self, p): ...
        def log_artifact(self, *a, **k): ...
        def end_run(self): ...

        def log_metrics(self, m, *, step=None):  # type: ignore[no-untyped-def]
            self.metrics.append((step, dict(m)))

    model = {"name": "gpt", "vocab_size": 32, "block_size": 8, "d_model": 64, "n_layers": 1, "n_heads": 2,
             "d_ff": 64, "dropout": 0.0, "extra": {"fused": fused}}
    cfg = RunConfig.model_validate(minimal_payload(
        model=model, ddp={"enabled": True},
        trainer={"max_steps": 4, "warmup_steps": 0, "micro_batch_size": 2, "grad_accum_steps": 2,
                 "log_every_steps": 2, "eval_every_steps": 4, "save_every_steps": 2},
    ))
    state = DDPState(rank=rank, world_size=world, local_rank=rank, is_main=rank == 0)
    rec = Recorder()
    run_dir = Path(out_dir) / "run" if rank == 0 else None
    result = Trainer(cfg, run_dir=run_dir, tracker=rec, ddp_state=state).fit()
    payload = {"metrics": rec.metrics, "final_loss": result.final_loss, "val": result.final_val_loss}
    (Path(out_dir) / f"rank{rank}.json").write_text(json.dumps(payload))
    dist.destroy_process_group()


@pytest.mark.parametrize("fused", [False, True])
def test_trainer_ddp_metrics_and_rank0_io(tmp_path: Path, fused: bool) -> None:
    mp.spawn(_trainer_worker, args=(2, _free_port(), str(tmp_path), fused), nprocs=2, join=True)
    r0 = json.loads((tmp_path / "rank0.json").read_text())
    r1 = json.loads((tmp_path / "rank1.json").read_text())
    assert r1["metrics"] == []  # only rank 0 logs
    keys = set().union(*(m for _, m in r0["metrics"]))
    for r in (0, 1):
        assert {f"train/loss_rank_{r}", f"train/tokens_per_sec_rank_{r}", f"val/loss_rank_{r}"} <= keys
    assert {"train/loss", "train/tokens_total", "val/loss"} <= keys
    assert [s for s, m in r0["metrics"] if "train/loss" in m] == [2, 4]
    ckpts = sorted(p.name for p in (tmp_path / "run" / "checkpoints").glob("*.pt"))
    assert ckpts == ["step_000002.pt", "step_000004.pt"]
    assert r0["val"] == pytest.approx(r1["val"])  # global val loss is the same on all ranks


def _dropout_stream_worker(rank: int, world: int, port: int, out_dir: str) -> None:
    _init(rank, world, port)
    from llmtrain.training.trainer import Trainer

    model = {"name": "gpt", "vocab_size": 32, "block_size": 8, "d_model": 64, "n_layers": 1, "n_heads": 2,
             "d_ff": 64, "dropout": 0.5, "extra": {"fused": True}}
    cfg = RunConfig.model_validate(minimal_payload(
        model=model, ddp={"enabled": True}, run={"name": "t", "seed": 11},
        trainer={"max_steps": 2, "warmup_steps": 0, "micro_batch_size": 2, "grad_accum_steps": 1},
    ))
    state = DDPState(rank=rank, world_size=world, local_rank=rank, is_main=rank == 0)
    tr = Trainer(cfg, ddp_state=state)
    params = torch.cat([p.detach().reshape(-1) for p in tr.model.parameters()])
    # the fused engine's per-forward dropout site seed and a module-path nn.Dropout mask
    site_seed = int(torch.randint(0, 2**31 - 1, (1,)).item())
    mask = torch.nn.functional.dropout(torch.ones(256), 0.5, training=True)
    torch.save({"params": params, "site_seed": site_seed, "mask": mask}, Path(out_dir) / f"drop{rank}.pt")
    dist.destroy_process_group()


def test_dropout_streams_differ_per_rank_but_init_is_shared(tmp_path: Path) -> None:
    mp.spawn(_dropout_stream_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "drop0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "drop1.pt", weights_only=True)
    assert torch.equal(r0["params"], r1["params"])
    assert r0["site_seed"] != r1["site_seed"]
    assert not torch.equal(r0["mask"], r1["mask"])


@pytest.mark.slow
def test_torchrun_cli_end_to_end(tmp_path: Path) -> None:
    cfg = yaml_safe_load(REPO / "configs" / "presets" / "ddp_smoke.yaml")
    cfg["output"]["root_dir"] = str(tmp_path / "runs")
    path = tmp_path / "ddp.yaml"
    import yaml

    path.write_text(yaml.safe_dump(cfg))
    env = dict(os.environ, PYTHONPATH=str(REPO), OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc_per_node=2", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), "-m", "llmtrain", "train", "--config", str(path), "--json"]
    proc = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert proc.returncode == 0, proc.stderr[-3000:]
    # stdout is exactly rank 0's JSON summary: libgloo's "[Gloo] Rank r is connected ..." lines
    # (written to fd 1 by the native library) land on stderr (cli._stdout_reserved)
    summary = json.loads(proc.stdout)
    assert summary["training"]["final_step"] == 10 and summary["ddp"]["env"]["WORLD_SIZE"] == "2"
    runs = list((tmp_path / "runs").iterdir())
    assert len(runs) == 1
    assert len(list((runs[0] / "checkpoints").glob("step_*.pt"))) == 10 // 10


def yaml_safe_load(path: Path) -> dict:
    import yaml

    return yaml.safe_load(path.read_text())
