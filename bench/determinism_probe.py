"""Find run-to-run variation in deterministic mode, step by step, inside one process.

    python bench/determinism_probe.py [--steps S] [--micro-batch B] [--reps R]
    python bench/determinism_probe.py --runs N [--steps S]      # whole runs, compared step by step

For each of S optimizer steps of GPT-2 124M (``run.deterministic: true``, fused engine, side
stream as configured by the environment) the forward + backward of that step's batch runs R times
from the SAME weights; every repetition's loss and flat gradient buffer must equal the first bit
for bit.  Then the optimizer steps with the last repetition's gradients and the next state is
probed.  A mismatch names the step, the repetition and every parameter whose gradient differs —
the kernel that produced it follows from the parameter (and the stream it ran on), which a
whole-run comparison at step 300 cannot tell.  One JSON line per mismatch, a summary line last.

``--runs N`` instead trains N fresh trainers (same seed, same data) for S steps exactly as
``Trainer.fit`` does — no host synchronisation between steps, so the CPU runs ahead and the
allocator sees the production free/reuse pattern — recording every step's loss and gradient norm
on the device; the runs must agree bit for bit at every step and in the final master weights, and
the first step where they do not is reported.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--micro-batch", type=int, default=32)
    ap.add_argument("--model", default="gpt2-124m")
    ap.add_argument("--dropout", type=float, default=0.0)
    ap.add_argument("--runs", type=int, default=0, help="compare N whole runs step by step instead")
    ap.add_argument("--pollute-gib", type=float, default=0.0,
                    help="--runs: before each run, fill this much freed device memory with a different "
                         "random pattern (a kernel that reads memory it never wrote shows up as a divergence)")
    args = ap.parse_args()

    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_main", Path(__file__).resolve().parents[1] / "bench.py")
    bench_mod = importlib.util.module_from_spec(spec)  # repo-root bench.py: the config builder
    spec.loader.exec_module(bench_mod)
    from llmtrain.training.trainer import Trainer, _to_device

    ns = argparse.Namespace(
        model=args.model, dropout=args.dropout, path="fused", device="cuda", deterministic=True,
        micro_batch=args.micro_batch, grad_accum=1, warmup=0, steps=args.steps, bucket_mb=64.0,
        grad_reduce_dtype="fp32", cuda_graph=False, backend="nccl",
    )
    torch.cuda.set_device(0)
    cfg = bench_mod.make_config(ns, 1)
    if args.runs:
        return compare_runs(cfg, args)
    trainer = Trainer(cfg)
    engine = trainer.model.engine
    store = engine.store
    names = {}
    for name, p in trainer.model.named_parameters():
        names[store.offset_of(p)] = (name, p.numel())
    stream = trainer.batch_stream()
    bad_total = 0
    t0 = time.perf_counter()
    # the Trainer scopes its kernel policy (run.deterministic) to train_step / fit; this loop
    # drives the engine directly, so it opens the same scope
    with trainer.kernel_policy():
        for step in range(1, args.steps + 1):
            batch = _to_device(stream.next(), trainer.device)
            ref_grad = ref_loss = None
            for rep in range(args.reps):
                trainer.optimizer.zero_grad()
                torch.manual_seed(1000 + step)  # the same dropout draw in every repetition
                with trainer._policy.autocast():
                    loss, _ = trainer._adapter.compute_loss(trainer.model, batch)
                loss.backward()
                torch.cuda.synchronize()
                if rep == 0:
                    ref_grad, ref_loss = store.grad.clone(), loss.detach().clone()
                    continue
                same_loss = bool(torch.equal(loss.detach(), ref_loss))
                if same_loss and torch.equal(store.grad, ref_grad):
                    continue
                bad_total += 1
                diff = store.grad != ref_grad
                params = []
                for off, (name, n) in sorted(names.items()):
                    cnt = int(diff[off : off + n].sum())
                    if cnt:
                        delta = float((store.grad[off : off + n] - ref_grad[off : off + n]).abs().max())
                        params.append({"param": name, "elems": cnt, "of": n, "max_abs": delta})
                print(json.dumps({"step": step, "rep": rep, "loss_equal": same_loss,
                                  "loss": [float(ref_loss), float(loss)], "params": params}), flush=True)
            trainer._optimizer_step()
            if step % 25 == 0:
                print(json.dumps({"progress": step, "elapsed_s": round(time.perf_counter() - t0, 1)}), flush=True)
    torch.cuda.synchronize()
    print(json.dumps({
        "summary": True, "steps": args.steps, "reps": args.reps, "micro_batch": args.micro_batch,
        "mismatches": bad_total, "wgrad_stream": os.environ.get("LLMTRAIN_WGRAD_STREAM", "0"),
        "tuned_table": bool(getattr(trainer, "tuned_gemms", False)),
        "master_checksum": float(store.master.double().sum()),
    }), flush=True)
    return 1 if bad_total else 0


def _pollute(gib: float, seed: int) -> None:
    """Hand the caching allocator ``gib`` GiB of freed blocks holding seed-dependent garbage (random
    floats, NaN and Inf patterns): the next run's buffers are carved from them, so a read of memory
    the run never wrote differs from run to run."""
    g = torch.Generator(device="cuda").manual_seed(1234 + seed)
    chunks = []
    for i in range(max(1, int(gib))):
        t = torch.empty(256 * 2**20, device="cuda")  # 1 GiB
        t.normal_(generator=g)
        if i % 4 == 1:
            t[seed::7] = float("nan")
        elif i % 4 == 3:
            t[seed::5] = float("inf")
        chunks.append(t)
    torch.cuda.synchronize()
    del chunks  # back to the allocator's free pool (no empty_cache)


def compare_runs(cfg, args: argparse.Namespace) -> int:  # type: ignore[no-untyped-def]
    from llmtrain.training.trainer import Trainer

    results = []
    for run in range(args.runs):
        t0 = time.perf_counter()
        if args.pollute_gib > 0:
            _pollute(args.pollute_gib, seed=run)
        trainer = Trainer(cfg)
        store = trainer.model.engine.store
        stream = trainer.batch_stream()
        losses, norms = [], []
        for _ in range(args.steps):
            loss, _ = trainer.train_step(stream)  # no host sync: the production issue pattern
            losses.append(loss.detach().reshape(1))
            norms.append(trainer.last_grad_norm.detach().reshape(1).float())
        torch.cuda.synchronize()
        results.append((torch.cat(losses).cpu(), torch.cat(norms).cpu(), store.master.clone()))
        print(json.dumps({"run": run, "final_loss": float(results[-1][0][-1]), "wall_s": round(time.perf_counter() - t0, 1),
                          "master_checksum": float(results[-1][2].double().sum())}), flush=True)
        del trainer, store, stream
        torch.cuda.empty_cache()
    bad = 0
    ref = results[0]
    for run, (lo, no, master) in enumerate(results[1:], start=1):
        diff = ((lo != ref[0]) | (no != ref[1])).nonzero().flatten()
        same_master = bool(torch.equal(master, ref[2]))
        if len(diff) or not same_master:
            bad += 1
        first = int(diff[0]) + 1 if len(diff) else None
        print(json.dumps({"run": run, "first_diverging_step": first, "diverging_steps": int(len(diff)),
                          "master_bitwise_equal": same_master,
                          "loss_at_first": None if first is None else [float(ref[0][first - 1]), float(lo[first - 1])],
                          "norm_at_first": None if first is None else [float(ref[1][first - 1]), float(no[first - 1])]}),
              flush=True)
    print(json.dumps({"summary": True, "mode": "runs", "runs": args.runs, "steps": args.steps,
                      "micro_batch": args.micro_batch, "runs_differing": bad,
                      "wgrad_stream": os.environ.get("LLMTRAIN_WGRAD_STREAM", "0")}), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
