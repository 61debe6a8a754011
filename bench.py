#!/usr/bin/env python3
"""Headline benchmark: GPT-2 124M training throughput on MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W            # N=1 directly
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W   # N>1, one rank per GPU (RCCL)

Each rank runs the real ``llmtrain`` Trainer (fused GPT engine, hand-written gfx950 kernels,
bucketed RCCL all-reduce, fused AdamW) on the reference GPT-2 124M architecture (V=50257,
T=1024, d=768, 12 layers, 12 heads, d_ff=3072, tied embeddings, random init) in bf16 with
synthetic token windows of the full block size.  W untimed warm-up steps, then EXACTLY K timed
optimizer steps (forward + backward + gradient all-reduce + clip + AdamW + LR schedule — nothing
skipped) bracketed by barrier + synchronize; the slowest rank's time counts.  Weak scaling: the
per-GPU batch is fixed, so the aggregate tokens/s is reported for the whole job.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_METRIC = "tokens/sec/GPU GPT-2-124M DDP at 1/2/4/8 MI355X; val-loss parity"

MODELS = {
    "gpt2-124m": dict(vocab_size=50257, block_size=1024, d_model=768, n_layers=12, n_heads=12, d_ff=3072),
    "gpt2-xl": dict(vocab_size=50257, block_size=1024, d_model=1600, n_layers=48, n_heads=25, d_ff=6400),
}


def make_config(args: argparse.Namespace, world: int):
    from llmtrain.config.schemas import RunConfig

    model = dict(MODELS[args.model], name="gpt", dropout=args.dropout, tie_embeddings=True)
    if args.path == "module":
        model["extra"] = {"fused": False}
    payload = {
        "schema_version": 1,
        "run": {"name": f"bench-{args.model}", "seed": 1337, "device": "cuda", "precision": "bf16"},
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
            "extra": {"bucket_cap_mb": args.bucket_mb},
        },
        "ddp": {"enabled": world > 1, "backend": "nccl"},
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
    ap.add_argument("--path", choices=["fused", "module"], default="fused")
    ap.add_argument("--dropout", type=float, default=0.0, help="model dropout (reference default 0.1)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    from llmtrain.parallel.dist import setup_ddp, teardown_ddp
    from llmtrain.training.trainer import Trainer

    cfg = make_config(args, world)
    ddp_state = None
    if world > 1:
        ddp_state = setup_ddp(cfg)
    else:
        torch.cuda.set_device(0)
    trainer = Trainer(cfg, ddp_state=ddp_state)
    batches = trainer.batch_stream()
    rank = ddp_state.rank if ddp_state else 0

    def barrier() -> None:
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        loss, _ = trainer.train_step(batches)
    barrier()
    t0 = time.perf_counter()
    tokens = 0
    for _ in range(args.steps):
        loss, n = trainer.train_step(batches)
        tokens += n
    barrier()
    elapsed = time.perf_counter() - t0
    final_loss = float(loss.item())
    want = args.steps * cfg.trainer.micro_batch_size * cfg.trainer.grad_accum_steps * cfg.model.block_size
    if tokens != want:  # a short data shard would silently shrink the per-GPU batch
        raise RuntimeError(f"rank {rank}: timed {tokens} tokens, expected {want}")

    elapsed_t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    tokens_t = torch.tensor([tokens], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(elapsed_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tokens_t, op=dist.ReduceOp.SUM)
    elapsed = float(elapsed_t.item())
    total_tokens = float(tokens_t.item())
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
            "dtype": "bf16",
            "data": "synthetic (seeded Markov token windows, full block_size), random-init weights",
            "config": {
                "model": "GPT-2 124M" if args.model == "gpt2-124m" else "GPT-2 XL 1.5B",
                "global_batch": global_batch,
                "seq_len": cfg.model.block_size,
                "parallelism": f"dp{world}",
                "micro_batch_per_gpu": cfg.trainer.micro_batch_size,
                "grad_accum": cfg.trainer.grad_accum_steps,
                "path": args.path,
                "dropout": args.dropout,
            },
            "tokens_per_sec_per_gpu": round(tps / world, 1),
            "mfu": round(mfu(tps / world, per_tok), 4),
            "final_loss": round(final_loss, 4),
            "peak_mem_gib": round(torch.cuda.max_memory_allocated() / 2**30, 2),
            "alloc_retries": int(torch.cuda.memory_stats().get("num_alloc_retries", 0)),
            "device_mallocs": int(torch.cuda.memory_stats().get("num_device_alloc", 0)),
            "reserved_gib": round(torch.cuda.memory_reserved() / 2**30, 2),
            "tuned_gemm_table": bool(getattr(trainer, "tuned_gemms", False)),
            "device_free_total_gib": [round(v / 2**30, 1) for v in torch.cuda.mem_get_info()],
        }
        print(json.dumps(result), flush=True)
    if ddp_state is not None:
        teardown_ddp()
    return 0


if __name__ == "__main__":
    sys.exit(main())
