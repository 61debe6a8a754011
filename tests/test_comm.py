"""Gradient-communication checks on CPU with real 2-process gloo worlds: the bf16-compressed bucket
path of the flat reducer against the fp32 one, the per-bucket timeline, the startup
all-reduce probe, and the parser of RCCL's transport log (reference: DDP Reducer buckets,
trainer.py:86-91; multi-process tests, tests/test_distributed.py:702-784)."""

from __future__ import annotations

import os
import socket
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from llmtrain.parallel import comm


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank: int, world: int, port: int) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)


def _grads_with(model, dtype, batch):  # type: ignore[no-untyped-def]
    from llmtrain.parallel.reducer import FlatDataParallel

    ddp = FlatDataParallel(model, bucket_cap_mb=0.02, reduce_dtype=dtype, broadcast_parameters=False)
    model.flat_store.zero_grad()
    ddp.fused_loss(batch, batch).backward()
    ddp.finish_gradient_sync()
    return model.flat_store.grad.clone(), ddp


def _bf16_worker(rank: int, world: int, port: int, out_dir: str) -> None:
    _init(rank, world, port)
    from llmtrain.models.gpt import GPT

    torch.manual_seed(7)  # same init on both ranks
    model = GPT(vocab_size=64, block_size=16, d_model=64, n_layers=2, n_heads=2, d_ff=128, dropout=0.0)
    model.prepare_runtime(compute_dtype=torch.float32)
    batch = torch.randint(0, 64, (2, 16), generator=torch.Generator().manual_seed(100 + rank))
    model.flat_store.zero_grad()
    model.fused_loss(batch, batch).backward()
    local = model.flat_store.grad.clone()
    g32, _ = _grads_with(model, None, batch)
    g16, ddp = _grads_with(model, torch.bfloat16, batch)
    steps = ddp.bucket_timeline()
    probe = comm.probe_allreduce(torch.device("cpu"), mib=1.0, iters=2, dtype=torch.float32)
    torch.save({"local": local, "g32": g32, "g16": g16, "nbuckets": len(ddp.buckets), "timeline": steps,
                "busbw": probe.busbw_gbps, "world": probe.world_size}, Path(out_dir) / f"r{rank}.pt")
    dist.destroy_process_group()


def test_bf16_bucket_reduce_matches_fp32(tmp_path: Path) -> None:
    mp.spawn(_bf16_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    mean = (r0["local"] + r1["local"]) / 2
    torch.testing.assert_close(r0["g32"], mean, atol=1e-7, rtol=1e-6)
    # bf16 on the wire: each rank's contribution is rounded to 8 significant bits before the sum
    # and the average is rounded again -> within ~2 bf16 ulps of the fp32 mean, everywhere
    err = (r0["g16"] - mean).abs()
    bound = 2 * 2.0**-8 * (r0["local"].abs() + r1["local"].abs()) / 2 + 1e-12
    assert bool((err <= bound + 2.0**-8 * mean.abs()).all()), float((err - bound).max())
    assert not torch.equal(r0["g16"], r0["g32"])  # the compressed path really ran
    assert torch.equal(r0["g16"], r1["g16"])  # every rank ends with the same gradient
    # one timeline row per bucket, host path: launch -> completion seen by the wait
    (steps,) = r0["timeline"]
    assert len(steps) == r0["nbuckets"] > 2
    assert all(row["ready_to_done_ms"] >= 0.0 and row["mib"] > 0 for row in steps)
    assert r0["busbw"] > 0 and r0["world"] == 2


def test_summarize_transport_counts_and_fallback(tmp_path: Path) -> None:
    log = tmp_path / "rccl.log"
    log.write_text(
        "host:1:1 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC comm 0x1 nRanks 02\n"
        "host:1:1 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC comm 0x1 nRanks 02\n"
        "host:1:1 [0] NCCL INFO 16 coll channels, 16 collnet channels, 0 nvls channels, 16 p2p channels\n"
    )
    s = comm.summarize_transport(log)
    assert s.counts == {"P2P": 2} and s.channels == 16 and not s.fallback and len(s.lines) == 3
    log.write_text("x NCCL INFO Channel 00 : 0[0] -> 1[1] via SHM/direct/direct\n")
    assert comm.summarize_transport(log).fallback
    assert comm.summarize_transport(tmp_path / "missing.log").counts == {}


def test_configure_rccl_env_respects_operator(monkeypatch: pytest.MonkeyPatch, tmp_path: Path) -> None:
    for key in ("NCCL_DEBUG", "NCCL_DEBUG_FILE", "NCCL_DEBUG_SUBSYS", "NCCL_MAX_NCHANNELS"):
        monkeypatch.delenv(key, raising=False)
    path = comm.configure_rccl_env({"transport_log_dir": str(tmp_path), "max_channels": 8}, rank=3)
    assert path is not None and "rank3" in path and os.environ["NCCL_DEBUG_FILE"] == path
    assert os.environ["NCCL_DEBUG"] == "INFO" and os.environ["NCCL_MAX_NCHANNELS"] == "8"
    monkeypatch.setenv("NCCL_DEBUG", "WARN")  # the operator's setting wins
    assert comm.configure_rccl_env({}, rank=0) is None and os.environ["NCCL_DEBUG"] == "WARN"


def test_rccl_debug_file_defaults_to_run_volume_and_relays_warnings(
    monkeypatch: pytest.MonkeyPatch, tmp_path: Path
) -> None:
    """NCCL_DEBUG_FILE swallows RCCL's warnings too: the file defaults to the run root (the PVC in
    Kubernetes, not the pod's /tmp) and its WARN lines are re-logged at startup / teardown."""
    for key in ("NCCL_DEBUG", "NCCL_DEBUG_FILE", "NCCL_DEBUG_SUBSYS"):
        monkeypatch.delenv(key, raising=False)
    path = comm.configure_rccl_env({}, rank=1, default_dir=tmp_path / "rccl")
    assert path is not None and Path(path).parent == tmp_path / "rccl"
    Path(path).write_text(
        "h:1:1 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC\n"
        "h:1:1 [0] NCCL WARN Call to ibv_open_device failed\n"
    )
    logged: list[str] = []
    monkeypatch.setattr(comm.logger, "warning", lambda fmt, *a: logged.append(fmt % a))
    assert comm.relay_warnings() == ["h:1:1 [0] NCCL WARN Call to ibv_open_device failed"]
    assert comm.relay_warnings() == []  # already relayed
    with open(path, "a") as fh:
        fh.write("h:1:1 [0] NCCL WARN watchdog timeout\n")
    assert comm.relay_warnings() == ["h:1:1 [0] NCCL WARN watchdog timeout"]
    assert sum("NCCL WARN" in line for line in logged) == 2
