#!/usr/bin/env python3
"""Headline benchmark: GPT-2 124M training throughput on MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W            # spawns N ranks itself when N > 1
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W   # or under an external launcher

With ``--gpus N > 1`` and no ``WORLD_SIZE`` in the environment, this process starts
``torch.distributed.run --nproc-per-node N`` as a CHILD process (before touching the GPU) and
exits with its code, so ``python bench.py --gpus 8`` really measures 8 RCCL ranks.  Every rank
asserts ``dist.get_world_size() == N`` and the ``nccl`` (= RCCL) backend.

Each rank runs the real ``llmtrain`` Trainer (fused GPT engine, hand-written gfx950 kernels,
bucketed RCCL all-reduce, fused AdamW) on the reference GPT-2 124M architecture (V=50257,
T=1024, d=768, 12 layers, 12 heads, d_ff=3072, tied embeddings, random init) in bf16 with
synthetic token windows of the full block size.  W untimed warm-up steps, then EXACTLY K timed
optimizer steps (forward + backward + gradient all-reduce + clip + AdamW + LR schedule — nothing
skipped) bracketed by barrier + synchronize; the slowest rank's time counts.  Weak scaling: the
per-GPU batch is fixed, so the aggregate tokens/s is reported for the whole job, plus per-rank
tokens/s and the exposed all-reduce time (communication not hidden behind the backward).

``--device cpu`` (gloo, fp32, ``--model tiny``) exists for the CPU contract tests only.
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_METRIC = "tokens/sec/GPU GPT-2-124M DDP at 1/2/4/8 MI355X; val-loss parity"

MODELS = {
    "gpt2-124m": dict(vocab_size=50257, block_size=1024, d_model=768, n_layers=12, n_heads=12, d_ff=3072),
    "gpt2-xl": dict(vocab_size=50257, block_size=1024, d_model=1600, n_layers=48, n_heads=25, d_ff=6400),
    "tiny": dict(vocab_size=512, block_size=64, d_model=64, n_layers=2, n_heads=2, d_ff=128),  # CPU tests
    # the reference presets' model shapes (configs/presets/*.yaml) with the GPT-2 vocabulary:
    # launch-bound on an MI355X, the case --cuda-graph is for
    "wikitext-better": dict(vocab_size=50257, block_size=256, d_model=384, n_layers=12, n_heads=8, d_ff=1536),
    "wikitext-ddp": dict(vocab_size=50257, block_size=256, d_model=256, n_layers=4, n_heads=4, d_ff=1024),
}
MODEL_LABEL = {"gpt2-124m": "GPT-2 124M", "gpt2-xl": "GPT-2 XL 1.5B", "tiny": "tiny (CPU contract test)",
               "wikitext-better": "gpt_wikitext_better shape (d 384, 12 layers)",
               "wikitext-ddp": "gpt_wikitext_ddp shape (d 256, 4 layers)"}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv: list[str]) -> int:
    """Run this script under ``torch.distributed.run`` with ``n`` local ranks (child process,
    never ``exec``: nothing here has touched the GPU yet) and return its exit code."""
    cmd = [
        sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv,
    ]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this driver
    env.setdefault("OMP_NUM_THREADS", "4")
    print(f"bench: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def summarize_buckets(steps: list[list[dict[str, float]]]) -> list[dict[str, float]]:
    """Mean per-bucket timeline over the timed steps (FlatDataParallel.bucket_timeline rows)."""
    if not steps:
        return []
    out = []
    for i in range(len(steps[0])):
        rows = [s[i] for s in steps if i < len(s)]
        summary: dict[str, float] = {"bucket": i, "payload_mib": rows[0]["mib"]}
        for key in ("ready_ms", "queue_ms", "comm_ms", "ready_to_done_ms"):
            vals = [r[key] for r in rows if key in r]
            if vals:
                summary[key] = round(sum(vals) / len(vals), 3)
        out.append(summary)
    return out


def make_config(args: argparse.Namespace, world: int):
    from llmtrain.config.schemas import RunConfig

    model = dict(MODELS[args.model], name="gpt", dropout=args.dropout, tie_embeddings=True)
    if args.path == "module":
        model["extra"] = {"fused": False}
    gpu = args.device == "cuda"
    if not gpu:
        model.setdefault("extra", {})["fused"] = args.path == "fused"
    residual = getattr(args, "residual", None)
    if args.path == "fused" and residual is not None:
        model.setdefault("extra", {})["residual_dtype"] = residual
    mlp_store = getattr(args, "mlp_store", None)
    if args.path == "fused" and mlp_store is not None:
        model.setdefault("extra", {})["mlp_store"] = mlp_store
    payload = {
        "schema_version": 1,
        # deterministic=False: the fast path's split-K / embedding atomics (run.deterministic
        # selects fixed-order reductions; synthetic data makes the data-order half moot)
        "run": {"name": f"bench-{args.model}", "seed": 1337, "device": args.device,
                "precision": "bf16" if gpu else "fp32", "deterministic": args.deterministic},
        "model": model,
        "data": {
            "name": "synthetic_tokens",
            "num_workers": 0,
            # every rank's DistributedSampler shard must hold whole micro-batches (8 ranks x 128)
            "extra": {"train_sequences": max(256, 4 * args.micro_batch * args.grad_accum * world), "val_sequences": 0},
        },
        "trainer": {
            "max_steps": args.warmup + args.steps + 1,
            "micro_batch_size": args.micro_batch,
            "grad_accum_steps": args.grad_accum,
            "lr": 6e-4,
            "weight_decay": 0.1,
            "warmup_steps": 0,
            "max_grad_norm": 1.0,
            "extra": {"bucket_cap_mb": args.bucket_mb, "grad_reduce_dtype": args.grad_reduce_dtype,
                      "cuda_graph": bool(getattr(args, "cuda_graph", False))},
        },
        "ddp": {"enabled": world > 1, "backend": getattr(args, "backend", "nccl") if gpu else "gloo"},
        "mlflow": {"enabled": False},
        "logging": {"log_to_file": False},
        "output": {"root_dir": "/tmp/llmtrain_bench_runs"},
    }
    return RunConfig.model_validate(payload)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", choices=sorted(MODELS), default="gpt2-124m")
    ap.add_argument("--micro-batch", type=int, default=128, help="sequences per GPU per micro-step")
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--grad-reduce-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="dtype of the gradient all-reduce payload (fused path)")
    ap.add_argument("--path", choices=["fused", "module"], default="fused")
    ap.add_argument("--dropout", type=float, default=0.0, help="model dropout (reference default 0.1)")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda", help="cpu: contract tests only")
    ap.add_argument("--deterministic", action="store_true", help="fixed-order reductions (run.deterministic)")
    ap.add_argument("--cuda-graph", action="store_true",
                    help="capture the optimizer step as a hipGraph and replay it (1 GPU, dropout 0)")
    ap.add_argument("--residual", choices=["fp32", "bf16_grad", "bf16"], default=None,
                    help="fused engine: storage of the residual stream / its gradient (model.extra.residual_dtype; "
                         "default: the engine's, bf16 with bf16 compute)")
    ap.add_argument("--mlp-store", choices=["u", "gd"], default=None,
                    help="fused engine: what the MLP keeps for its backward (model.extra.mlp_store)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="gloo on GPU: rehearse the N-rank path on a box with fewer GPUs (ranks share devices)")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2
    gpu = args.device == "cuda"
    from llmtrain.parallel.comm import last_probe
    from llmtrain.parallel.dist import setup_ddp, teardown_ddp
    from llmtrain.training.trainer import Trainer

    cfg = make_config(args, world)
    ddp_state = None
    if world > 1:
        ddp_state = setup_ddp(cfg)
        got_world, backend = dist.get_world_size(), dist.get_backend()
        want_backend = args.backend if gpu else "gloo"
        if got_world != args.gpus or backend != want_backend:
            raise RuntimeError(f"rank {ddp_state.rank}: world={got_world} backend={backend}, "
                               f"expected world={args.gpus} backend={want_backend}")
    elif gpu:
        torch.cuda.set_device(0)
    trainer = Trainer(cfg, ddp_state=ddp_state)
    batches = trainer.batch_stream()
    rank = ddp_state.rank if ddp_state else 0
    dev = torch.device("cuda", torch.cuda.current_device()) if gpu else torch.device("cpu")
    drain = getattr(trainer.model, "drain_exposed_comm_ms", None)
    timeline = getattr(trainer.model, "bucket_timeline", None)

    def barrier() -> None:
        if world > 1:
            dist.barrier()
        if gpu:
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        loss, _ = trainer.train_step(batches)
    barrier()
    if drain is not None:
        drain()
    if timeline is not None:
        timeline()
    t0 = time.perf_counter()
    tokens = 0
    for _ in range(args.steps):
        loss, n = trainer.train_step(batches)
        tokens += n
    barrier()
    elapsed = time.perf_counter() - t0
    final_loss = float(loss.item())
    comm = drain() if drain is not None else []
    comm_ms = sum(comm) / len(comm) if comm else 0.0
    buckets = summarize_buckets(timeline() if timeline is not None else [])
    want = args.steps * cfg.trainer.micro_batch_size * cfg.trainer.grad_accum_steps * cfg.model.block_size
    if tokens != want:  # a short data shard would silently shrink the per-GPU batch
        raise RuntimeError(f"rank {rank}: timed {tokens} tokens, expected {want}")

    mine = torch.tensor([elapsed, float(tokens), comm_ms], dtype=torch.float64, device=dev)
    if world > 1:
        gathered = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(gathered, mine)
    else:
        gathered = [mine]
    rows = [g.tolist() for g in gathered]
    elapsed = max(r[0] for r in rows)
    total_tokens = sum(r[1] for r in rows)
    tps = total_tokens / elapsed
    if rank == 0:
        from llmtrain.utils.flops import mfu, training_flops_per_token

        raw = getattr(trainer.model, "module", trainer.model)
        per_tok = training_flops_per_token(raw, cfg.model.block_size)
        global_batch = cfg.trainer.micro_batch_size * cfg.trainer.grad_accum_steps * world
        result = {
            "metric": BASELINE_METRIC,
            "value": round(tps, 1),
            "unit": "tokens/s (aggregate over all GPUs)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if gpu else "fp32",
            "data": "synthetic (seeded Markov token windows, full block_size), random-init weights",
            "config": {
                "model": MODEL_LABEL[args.model],
                "global_batch": global_batch,
                "seq_len": cfg.model.block_size,
                "parallelism": f"dp{world}",
                "micro_batch_per_gpu": cfg.trainer.micro_batch_size,
                "grad_accum": cfg.trainer.grad_accum_steps,
                "path": args.path,
                "dropout": args.dropout,
                "grad_reduce_dtype": args.grad_reduce_dtype,
                "deterministic": args.deterministic,
                "backend": dist.get_backend() if world > 1 else None,
                "cuda_graph": bool(args.cuda_graph),
                "residual_dtype": getattr(getattr(raw, "engine", None), "residual", None),
                "mlp_store": getattr(getattr(raw, "engine", None), "mlp_store", None),
            },
            "tokens_per_sec_per_gpu": round(tps / world, 1),
            "per_rank_tokens_per_sec": [round(r[1] / r[0], 1) for r in rows],
            "exposed_allreduce_ms": [round(r[2], 3) for r in rows],
            "value_semantics": "value = aggregate tokens/s of the whole job (all ranks); per GPU: tokens_per_sec_per_gpu",
            "final_loss": round(final_loss, 4),
        }
        if gpu:
            result.update({
                "mfu": round(mfu(tps / world, per_tok), 4),
                "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 2),
                "alloc_retries": int(torch.cuda.memory_stats().get("num_alloc_retries", 0)),
                "device_mallocs": int(torch.cuda.memory_stats().get("num_device_alloc", 0)),
                "reserved_gib": round(torch.cuda.memory_reserved() / 2**30, 2),
                "tuned_gemm_table": bool(getattr(trainer, "tuned_gemms", False)),
                "device_free_total_gib": [round(v / 2**30, 1) for v in torch.cuda.mem_get_info()],
            })
        probe = last_probe()
        if probe is not None:
            result["allreduce_busbw_gbps"] = round(probe.busbw_gbps, 1)
            result["allreduce_probe"] = {k: (round(v, 3) if isinstance(v, float) else v)
                                         for k, v in probe.as_dict().items()}
            for b in buckets:  # what the bucket would take alone at the probed bus bandwidth
                b["alone_ms"] = round(b["payload_mib"] * 2**20 * 2 * (world - 1) / world / probe.busbw_gbps / 1e6, 3)
        if world > 1:  # the first multi-GPU run has to explain itself (channels, transports)
            from llmtrain.parallel.comm import rccl_report

            result["rccl"] = rccl_report()
        if buckets:
            result["buckets_rank0"] = buckets
            # the last bucket (the tied embedding, final in the backward) cannot overlap compute:
            # its queue + collective time is what the step exposes
            tail = buckets[-1]
            result["tail_bucket"] = {k: tail[k] for k in ("bucket", "payload_mib", "queue_ms", "comm_ms", "alone_ms")
                                     if k in tail}
        print(json.dumps(result), flush=True)
    if ddp_state is not None:
        teardown_ddp()
    return 0


if __name__ == "__main__":
    sys.exit(main())
