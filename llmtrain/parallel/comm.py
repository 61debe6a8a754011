"""Startup checks of the data-parallel transport: RCCL environment, transport log, bus bandwidth.

The reference's DDP runs on gloo over TCP and never checks what it got
(``distributed/__init__.py:130-136``).  On an 8 x MI355X node the gradient all-reduce must ride
RCCL's peer-to-peer path over the xGMI links (7 links x ~153 GB/s per GPU); a pod layout that
hides the peer GPUs silently drops RCCL to shared memory or sockets, which would
show up only as a bad scaling number.  Three checks make it visible at startup:

* :func:`configure_rccl_env` (before ``init_process_group``): RCCL's INIT/GRAPH debug lines go to a
  per-rank file (``NCCL_DEBUG_FILE``) instead of stderr — unless the operator set ``NCCL_DEBUG``
  themselves — and the optional channel budget (``ddp.extra.max_channels`` / ``min_channels`` →
  ``NCCL_MAX_NCHANNELS`` / ``NCCL_MIN_NCHANNELS``: one workgroup per channel, i.e. the CUs RCCL
  takes from the compute streams while a bucket is in flight);
* :func:`probe_allreduce` (after it): a few large bf16 all-reduces on the real process group,
  reported as bus bandwidth (``2(n-1)/n · bytes / time``, the per-link figure a ring moves);
* :func:`summarize_transport`: the transports RCCL connected its channels with (``P2P``,
  ``SHM``, ``NET``), parsed from that file and logged on rank 0 together with the raw lines.

``ddp.extra.min_busbw_gbps`` turns a low bandwidth from a warning into an error.
"""

from __future__ import annotations

import logging
import os
import re
import tempfile
import time
from dataclasses import asdict, dataclass, field
from pathlib import Path
from typing import Any

import torch
import torch.distributed as dist

__all__ = [
    "BusBandwidth",
    "TransportSummary",
    "check_transport",
    "configure_rccl_env",
    "current_transport",
    "last_probe",
    "probe_allreduce",
    "rccl_report",
    "relay_warnings",
    "summarize_transport",
]

logger = logging.getLogger(__name__)

# xGMI: ~153 GB/s per link; a healthy 8-GPU RCCL all-reduce of 256 MiB reaches well over one link
# of bus bandwidth.  Below this a warning names the likely cause (SHM / socket fallback).
WARN_BUSBW_GBPS = 40.0

_TRANSPORT_RE = re.compile(r"via (P2P(?:/[\w.]+)?|SHM(?:/[\w.]+)*|NET/[\w.]+|COLLNET\S*)")
_CHANNELS_RE = re.compile(r"(\d+) coll channels")

_state: dict[str, Any] = {"probe": None, "debug_file": None, "relayed": 0}


@dataclass(frozen=True)
class BusBandwidth:
    world_size: int
    bytes: int
    iters: int
    ms_per_iter: float
    algbw_gbps: float
    busbw_gbps: float
    dtype: str
    backend: str

    def as_dict(self) -> dict[str, Any]:
        return asdict(self)


@dataclass
class TransportSummary:
    counts: dict[str, int] = field(default_factory=dict)  # "P2P" / "SHM" / "NET" -> connection lines
    channels: int | None = None
    lines: list[str] = field(default_factory=list)

    @property
    def fallback(self) -> bool:
        """True when any channel connected through shared memory or the network stack."""
        return any(self.counts.get(k, 0) for k in ("SHM", "NET"))


def configure_rccl_env(extra: dict[str, Any], rank: int, default_dir: str | os.PathLike[str] | None = None) -> str | None:
    """Set RCCL environment knobs before the process group exists; returns the debug-file path
    (None when the operator owns ``NCCL_DEBUG`` or ``ddp.extra.log_transport`` is false).

    The file lives under ``ddp.extra.transport_log_dir``, else ``default_dir`` (the run's
    ``output.root_dir``/``rccl``: on the runs PVC in Kubernetes, so it outlives the pod), else the
    temp directory.  ``NCCL_DEBUG_FILE`` takes ALL of RCCL's output, warnings included, so
    :func:`relay_warnings` copies its ``WARN`` lines to the log (stderr) at startup and teardown."""
    for key, env in (("max_channels", "NCCL_MAX_NCHANNELS"), ("min_channels", "NCCL_MIN_NCHANNELS")):
        if extra.get(key) is not None:
            os.environ[env] = str(int(extra[key]))
    _state["debug_file"] = None
    if not bool(extra.get("log_transport", True)) or "NCCL_DEBUG" in os.environ:
        return None
    root = Path(extra.get("transport_log_dir") or default_dir or tempfile.gettempdir())
    try:
        root.mkdir(parents=True, exist_ok=True)
    except OSError:
        root = Path(tempfile.gettempdir())
    path = root / f"llmtrain-rccl-rank{rank}-{os.getpid()}.log"
    _state["relayed"] = 0
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,GRAPH")
    os.environ["NCCL_DEBUG_FILE"] = str(path)
    _state["debug_file"] = str(path)
    return str(path)


def summarize_transport(path: str | os.PathLike[str] | None, *, keep_lines: int = 24) -> TransportSummary:
    """Transport counts and channel count from an RCCL INIT/GRAPH debug file (missing file: empty)."""
    summary = TransportSummary()
    if path is None or not Path(path).exists():
        return summary
    for line in Path(path).read_text(errors="replace").splitlines():
        m = _TRANSPORT_RE.search(line)
        if m:
            kind = m.group(1).split("/")[0]
            summary.counts[kind] = summary.counts.get(kind, 0) + 1
            if len(summary.lines) < keep_lines:
                summary.lines.append(line.strip())
        c = _CHANNELS_RE.search(line)
        if c:
            summary.channels = int(c.group(1))
            if len(summary.lines) < keep_lines:
                summary.lines.append(line.strip())
    return summary


def relay_warnings(path: str | os.PathLike[str] | None = None) -> list[str]:
    """Log (WARNING, to stderr) every ``WARN`` line RCCL wrote to its debug file since the last
    call — transport errors and watchdog timeouts would otherwise only be in that file."""
    path = path or _state["debug_file"]
    if path is None or not Path(path).exists():
        return []
    lines = Path(path).read_text(errors="replace").splitlines()
    start = int(_state.get("relayed") or 0)
    _state["relayed"] = len(lines)
    warns = [ln.strip() for ln in lines[start:] if " WARN " in ln or "NCCL WARN" in ln]
    for ln in warns:
        logger.warning("rccl: %s", ln)
    return warns


def _sync(device: torch.device) -> None:
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def probe_allreduce(
    device: torch.device, *, mib: float = 256.0, iters: int = 3, dtype: torch.dtype = torch.bfloat16, group: Any = None
) -> BusBandwidth:
    """Time ``iters`` all-reduces of a ``mib`` MiB tensor (after one untimed warm-up that also
    creates the communicator); every rank gets the slowest rank's time."""
    world = dist.get_world_size(group)
    elem = torch.empty((), dtype=dtype).element_size()
    n = max(1, int(mib * 2**20) // elem)
    buf = torch.ones(n, dtype=dtype, device=device)
    dist.all_reduce(buf, group=group)  # warm-up + lazy communicator init
    _sync(device)
    dist.barrier(group=group)
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(buf, group=group)
    _sync(device)
    elapsed = time.perf_counter() - t0
    worst = torch.tensor([elapsed], dtype=torch.float64, device=device if device.type == "cuda" else "cpu")
    dist.all_reduce(worst, op=dist.ReduceOp.MAX, group=group)
    sec = float(worst.item()) / iters
    nbytes = n * elem
    algbw = nbytes / sec / 1e9
    busbw = algbw * (2.0 * (world - 1) / world if world > 1 else 1.0)
    result = BusBandwidth(
        world_size=world, bytes=nbytes, iters=iters, ms_per_iter=1000.0 * sec, algbw_gbps=algbw, busbw_gbps=busbw,
        dtype=str(dtype).replace("torch.", ""), backend=str(dist.get_backend(group)),
    )
    _state["probe"] = result
    return result


def current_transport() -> TransportSummary:
    """:func:`summarize_transport` of this process's RCCL debug file (empty without one)."""
    return summarize_transport(_state["debug_file"])


def rccl_report() -> dict[str, Any]:
    """What a multi-GPU result needs to explain itself: the transports RCCL connected its channels
    with, the channel count, whether any fell back to SHM / NET, and the channel / algorithm env
    knobs in force (``ddp.extra.max_channels`` etc.)."""
    t = current_transport()
    env = {k: os.environ[k] for k in ("NCCL_MAX_NCHANNELS", "NCCL_MIN_NCHANNELS", "NCCL_ALGO", "NCCL_PROTO")
           if k in os.environ}
    return {"transport_counts": dict(t.counts), "channels": t.channels, "fallback": t.fallback, "env": env,
            "debug_file": _state["debug_file"]}


def last_probe() -> BusBandwidth | None:
    """The result of the most recent :func:`probe_allreduce` in this process (None before)."""
    return _state["probe"]


def check_transport(device: torch.device, extra: dict[str, Any], *, rank: int) -> BusBandwidth | None:
    """Run the startup probe and the transport summary; log both on rank 0, warn (or raise under
    ``ddp.extra.min_busbw_gbps``) when the bandwidth is low or RCCL fell back to SHM/NET."""
    mib = float(extra.get("probe_allreduce_mib", 256.0 if device.type == "cuda" else 0.0))
    probe = None
    if mib > 0:
        probe = probe_allreduce(device, mib=mib, iters=int(extra.get("probe_iters", 3)))
        if rank == 0:
            logger.info(
                "ddp/allreduce_busbw_gbps=%.1f (algbw %.1f GB/s, %.1f MiB %s x %d ranks, %.3f ms, backend %s)",
                probe.busbw_gbps, probe.algbw_gbps, probe.bytes / 2**20, probe.dtype, probe.world_size,
                probe.ms_per_iter, probe.backend,
            )
    summary = summarize_transport(_state["debug_file"])
    relay_warnings()
    if rank == 0 and (summary.counts or summary.channels is not None):
        logger.info("rccl transport: %s channels=%s", summary.counts, summary.channels)
        for line in summary.lines:
            logger.info("rccl: %s", line)
    floor = extra.get("min_busbw_gbps")
    if probe is not None and probe.backend == "nccl":
        if floor is not None and probe.busbw_gbps < float(floor):
            raise RuntimeError(
                f"all-reduce bus bandwidth {probe.busbw_gbps:.1f} GB/s is below ddp.extra.min_busbw_gbps={floor}"
                f" (transports {summary.counts or 'unknown'})"
            )
        if probe.world_size > 1 and (probe.busbw_gbps < WARN_BUSBW_GBPS or summary.fallback):
            logger.warning(
                "all-reduce bus bandwidth %.1f GB/s with transports %s: RCCL is likely not on xGMI P2P "
                "(peer GPUs hidden from this process? see docs/k8s.md)", probe.busbw_gbps, summary.counts,
            )
    return probe
