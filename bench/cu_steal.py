"""How much does a training step lose when a concurrent kernel holds some CUs?

At N > 1 GPUs the gradient all-reduce (RCCL, one workgroup per channel) runs on a side stream
while the backward's GEMMs run.  Our GEMMs size their grids for the whole chip: the fused GEMM is
persistent (one workgroup per CU) and the weight-gradient planner fills one round of the CUs, so
a workgroup that finds its CU taken waits for a whole other workgroup's lifetime.  This probe
stands a CU thief in for the collective: `blocks` one-wave workgroups on a second stream stay
resident for the whole timed run (bench/native/cu_spin.cpp; a worst case — a real
collective holds its CUs for its own duration only), and the step time is compared with none.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC bench/native/cu_spin.cpp -o bench/native/bin/libcu_spin.so
    python bench/cu_steal.py --blocks 0 8 16 32 [--micro-batch 128]
"""

from __future__ import annotations

import argparse
import ctypes
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--blocks", type=int, nargs="+", default=[0, 8, 16, 32])
    ap.add_argument("--model", default="gpt2-124m")
    ap.add_argument("--micro-batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--thief-ms", type=float, default=0.0,
                    help="thief lifetime; 0: 2.5 x the free run measured first (skipped when given)")
    args = ap.parse_args()

    import bench as B  # the repo-root bench.py: its config builder

    lib = ctypes.CDLL(str(ROOT / "bench/native/bin/libcu_spin.so"))
    lib.llmt_cu_spin.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_void_p]
    lib.llmt_cu_spin.restype = ctypes.c_int

    from llmtrain.training.trainer import Trainer

    ns = argparse.Namespace(gpus=1, steps=args.steps, warmup=args.warmup, model=args.model,
                            micro_batch=args.micro_batch, grad_accum=1, bucket_mb=64.0, grad_reduce_dtype="fp32",
                            path="fused", dropout=0.0, device="cuda", deterministic=False, cuda_graph=False,
                            residual=None, mlp_store=None, backend="nccl")
    cfg = B.make_config(ns, 1)
    torch.cuda.set_device(0)
    trainer = Trainer(cfg, ddp_state=None)
    batches = trainer.batch_stream()
    side = torch.cuda.Stream(priority=-1)

    main_stream = torch.cuda.current_stream()

    def run(blocks: int, ticks: int) -> float:
        torch.cuda.synchronize()
        if blocks:  # one thief for the whole timed run; only the main stream is waited on
            rc = lib.llmt_cu_spin(blocks, ticks, ctypes.c_void_p(side.cuda_stream))
            if rc:
                raise RuntimeError(f"cu_spin launch failed: {rc}")
        t0 = time.perf_counter()
        for _ in range(args.steps):
            trainer.train_step(batches)
        main_stream.synchronize()
        ms = 1000.0 * (time.perf_counter() - t0) / args.steps
        torch.cuda.synchronize()  # drain the thief before the next arm
        return ms

    for _ in range(args.warmup):
        trainer.train_step(batches)
    base = run(0, 0) if args.thief_ms <= 0 else 0.0
    # 100 MHz clock: 2.5 x the free run (capped at 3 s)
    ticks = int((args.thief_ms if args.thief_ms > 0 else base * args.steps * 2.5) * 1e5)
    for r in range(args.rounds):
        for blocks in args.blocks:
            ms = run(blocks, ticks)
            print(json.dumps({"round": r, "blocks": blocks, "ms_per_step": round(ms, 2),
                              "vs_free": round(ms / base, 4) if base else None, "free_ms": round(base, 2)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
