"""Headline benchmark: whole-node training tokens/sec, GPT-2 124M bf16 DDP.

BASELINE.json metric/config: GPT-2 124M, nanoGPT ``train_gpt2`` semantics —
480 sequences x 1024 tokens = 491,520 tokens per optimizer step regardless of
N (strong scaling of a fixed global batch), synthetic tokens, random init.
nanoGPT reaches that batch as micro-batch 12 x 40 accumulation steps because
an A100 has 40 GB; on a 288 GB MI355X the same global batch runs as fewer,
larger micro-steps (auto: the largest divisor of 480/N that is <= 120, i.e.
120 x 4 on one GPU, 60 x 1 per rank on eight).  ``--micro-batch 12``
reproduces nanoGPT's exact schedule.  One timed "step" is a full
optimizer iteration: grad_accum x (fwd + bwd) with the bucketed RCCL
all-reduce overlapped on the last micro-step, global-norm clip, fused AdamW.

    python bench.py --gpus 1 --steps 5 --warmup 2
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8 --steps 10 --warmup 3

Rank 0 prints exactly one JSON line on stdout (everything else goes to stderr).
"""

from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

import torch
import torch.distributed as dist

GLOBAL_MICRO_STEPS = 40  # nanoGPT train_gpt2: 5 * 8
METRIC = "tokens/sec (whole node) GPT-2 124M DDP"


def batch_plan(world: int, micro_batch: int = 0) -> tuple[int, int]:
    """(micro-batch per rank, global micro-step count) for nanoGPT's fixed 480-sequence step.

    Auto (micro_batch <= 0): the largest divisor of the per-rank batch (480/world
    sequences) that is <= 120.  The global micro-step count is what the Trainer
    takes as ``gradient_accumulation_steps`` (nanoGPT divides it by world size),
    so micro_batch * total_micro == 480 for every world size.
    """
    global_seqs = GLOBAL_MICRO_STEPS * 12  # nanoGPT: 12 x 40 = 480 sequences per step
    assert global_seqs % world == 0, "global batch must divide over the ranks"
    per_rank_seqs = global_seqs // world
    if micro_batch <= 0:
        micro_batch = max(d for d in range(1, 121) if per_rank_seqs % d == 0)
    assert per_rank_seqs % micro_batch == 0, "micro-batch must divide the per-rank batch"
    return micro_batch, per_rank_seqs // micro_batch * world


def rccl_summary(report, sweep, reducer=None, exposed=None, early=None) -> dict | None:
    """The JSON record's RCCL block (None on one GPU).

    With the flat reducer it also carries the bucket layout (sizes, which parameters share
    the late embedding tail) and, per timed step, the exposed communication: the time the
    compute stream waited in ``reducer.finish()`` after the last backward kernel
    (``exposed_allreduce_ms``, max over ranks), plus how many buckets were launched while
    the backward was still running."""
    if not report and not sweep and reducer is None:
        return None
    report = report or {}
    out = {"backend": report.get("backend"), "preset": report.get("preset"),
           "transport_by_rank": {str(k): v for k, v in (report.get("transport") or {}).items()},
           "allreduce_64MiB_ms": report.get("allreduce_ms"), "allreduce_64MiB_busbw_GBps": report.get("busbw_GBps"),
           "sweep": list(sweep or [])}
    if reducer is not None:
        out["buckets"] = reducer.layout()
        out["exposed_allreduce_ms"] = round(sum(exposed) / len(exposed), 3) if exposed else None
        out["exposed_allreduce_ms_per_step"] = [round(v, 3) for v in (exposed or [])]
        out["buckets_launched_in_backward"] = list(early or [])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--micro-batch", type=int, default=0,
                    help="sequences per micro-step; 0 = auto: the largest divisor of the per-rank "
                         "batch (480/N sequences) that is <= 120 (uses MI355X's 288 GB instead of "
                         "nanoGPT's A100-sized 12; the 491,520-token global batch is unchanged)")
    ap.add_argument("--block-size", type=int, default=1024)
    ap.add_argument("--model", default="gpt2", choices=["gpt2", "gpt2-medium", "gpt2-large", "gpt2-xl", "tiny"],
                    help="tiny (2 x 64): plumbing tests of the multi-rank path only, not a benchmark")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: gloo rehearsal of the N > 1 path (tests/test_bench_plan.py), not a benchmark")
    ap.add_argument("--ddp-impl", default="flat", choices=["flat", "torch"])
    ap.add_argument("--bucket-mb", type=int, default=64)
    ap.add_argument("--grad-ckpt", action="store_true")
    ap.add_argument("--recompute-mlp", action="store_true",
                    help="selective recomputation: each MLP keeps only its input and recomputes c_fc + GELU in "
                         "the backward (config key recompute_mlp)")
    ap.add_argument("--bias", action="store_true",
                    help="Linear / LayerNorm biases (nanoGPT bias=True, the GPT-2 checkpoints' layout)")
    ap.add_argument("--deterministic", action="store_true",
                    help="bitwise-reproducible step: fixed-order split-K weight gradients, sorted embedding "
                         "backward, ordered LayerNorm dW/db (no fp32 atomics)")
    ap.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "float16"],
                    help="compute dtype (nanoGPT's dtype key): float16 runs the fp16 instantiation of every "
                         "kernel with the dynamic loss scale on the device (the headline is bfloat16)")
    ap.add_argument("--bf16-residual", action="store_true",
                    help="keep the residual stream and its gradient in bf16 (default fp32: nanoGPT's "
                         "autocast contract, fp32 embedding sum and fp32 + bf16 residual adds)")
    ap.add_argument("--real-data", default="",
                    help="dataset name or directory with train.bin/val.bin (nanoGPT bench.py real_data); "
                         "default: synthetic uniform tokens")
    ap.add_argument("--rccl-sweep", default="4,16,64,256",
                    help="all-reduce sizes (MiB) timed once before the timed steps when WORLD_SIZE > 1 "
                         "(bus bandwidth by bucket size, printed to stderr); '' disables")
    ap.add_argument("--calib-seconds", type=float, default=2.0,
                    help="box calibration after the timed steps: our NT GEMM on a fixed shape for this many "
                         "seconds (TF/s in the record's 'box' block, with the sclk/mclk DPM levels read before "
                         "and after the timed loop); 0 disables")
    ap.add_argument("--per-rank-of", type=int, default=0, metavar="N",
                    help="PROJECTION (not the headline): run one rank's share of an N-GPU job on this one GPU "
                         "-- the N-rank micro-batch plan (60 x 1 at N = 8), the flat reducer's hooks armed, each "
                         "bucket all-reduce replaced by a collective-shaped kernel on a high-priority side stream "
                         "for its modelled ring time (parallel/emulate.py) -- and report the per-rank step and "
                         "the projected N-GPU tokens/s")
    ap.add_argument("--emu-busbw", type=float, default=300.0,
                    help="--per-rank-of: assumed RCCL all-reduce bus bandwidth, GB/s (not measured here)")
    ap.add_argument("--emu-nwg", type=int, default=32,
                    help="--per-rank-of: workgroups of the emulated collective kernel (RCCL channels)")
    ap.add_argument("--profile", action="store_true",
                    help="nanoGPT bench.py profile mode: torch.profiler over the timed steps "
                         "(schedule wait 1 / warmup 1 / active rest), TensorBoard trace under ./bench_log")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    emu = args.per_rank_of if args.per_rank_of > 1 else 0
    if emu and (world != 1 or args.device != "cuda"):
        raise SystemExit("--per-rank-of runs one process on one GPU")
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("for --gpus > 1 launch with: python -m torch.distributed.run --nproc-per-node N bench.py ...")
        raise SystemExit(f"--gpus {args.gpus} does not match WORLD_SIZE {world}")

    from nanosandbox_amd.config import TRAIN_DEFAULTS
    from nanosandbox_amd.train import Trainer

    dims = {"gpt2": (12, 12, 768), "gpt2-medium": (24, 16, 1024), "gpt2-large": (36, 20, 1280),
            "gpt2-xl": (48, 25, 1600), "tiny": (2, 2, 64)}[args.model]
    cuda = args.device == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize()

    if args.micro_batch <= 0 and not args.grad_ckpt and not args.recompute_mlp and cuda:
        # HBM-sized micro-batch: the largest divisor of the per-rank batch whose activations
        # stay resident next to the model state (utils/memory.py); 120 for GPT-2 124M / 350M
        from nanosandbox_amd.utils.memory import choose_micro_batch
        # every rank of a one-GPU rehearsal (NSA_REHEARSAL_ONE_GPU, parallel/dist.py) runs on cuda:0
        dev_index = 0 if os.environ.get("NSA_REHEARSAL_ONE_GPU") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
        hbm = torch.cuda.get_device_properties(dev_index).total_memory
        if os.environ.get("NSA_REHEARSAL_ONE_GPU") == "1":
            hbm //= world  # the ranks share the one GPU's HBM
        args.micro_batch, _ = choose_micro_batch(dims[0], dims[2], dims[1], 50304, args.block_size,
                                                 480 // (emu or world), hbm, fp32_residual=not args.bf16_residual)
    args.micro_batch, total_micro = batch_plan(emu or world, args.micro_batch)
    if emu:
        total_micro //= emu  # this process runs one rank's micro-steps (the Trainer's world is 1)
    tokens_per_micro = args.micro_batch * args.block_size
    cfg = dict(TRAIN_DEFAULTS)
    dataset, data_dir = "synthetic", ""
    if args.real_data:
        if os.path.isdir(args.real_data):
            dataset, data_dir = os.path.basename(os.path.normpath(args.real_data)), args.real_data
        else:
            dataset = args.real_data
    cfg.update(dataset=dataset, data_dir=data_dir, batch_size=args.micro_batch, block_size=args.block_size,
               gradient_accumulation_steps=total_micro, n_layer=dims[0], n_head=dims[1], n_embd=dims[2],
               dropout=0.0, bias=args.bias, compile=False, device=args.device, dtype=args.dtype,
               backend="nccl" if cuda else "gloo",
               ddp_impl=args.ddp_impl, ddp_bucket_mb=args.bucket_mb, grad_ckpt=args.grad_ckpt,
               recompute_mlp=args.recompute_mlp,
               fp32_residual=not args.bf16_residual, deterministic=args.deterministic,
               out_dir="/tmp/nsa_bench_out", metrics_jsonl=False, learning_rate=6e-4, warmup_iters=0,
               decay_lr=False)

    with contextlib.redirect_stdout(sys.stderr):
        tr = Trainer(cfg)
        if emu:
            from nanosandbox_amd.parallel.emulate import EmulatedAllReduce
            tr.reducer = EmulatedAllReduce(tr.store, emu, bucket_cap_mb=args.bucket_mb, busbw_GBps=args.emu_busbw,
                                           nwg=args.emu_nwg)
            print(f"per-rank-of {emu}: {tr.gas} micro-step(s) of {args.micro_batch} x {args.block_size}, "
                  f"emulated all-reduce {json.dumps(tr.reducer.model())}")
        for g in tr.optimizer.param_groups:
            g["lr"] = cfg["learning_rate"]
        X, Y = tr.batches.get_batch("train")
        for _ in range(args.warmup):
            loss, _, X, Y = tr.train_step(X, Y)
        from nanosandbox_amd.ops import gemm_dispatch
        gemm_kernels = {f"{k[0]} {k[1]}x{k[2]}x{k[3]}": v for k, v in sorted(gemm_dispatch.kernels_used().items())}
        for k, v in gemm_kernels.items():
            print(f"gemm {k}: {v}")
        sweep = []
        if world > 1 and args.rccl_sweep:
            from nanosandbox_amd.parallel import allreduce_sweep
            sweep = allreduce_sweep(tr.info, [int(v) for v in args.rccl_sweep.split(",") if v])
        multi = dist.is_initialized() and world > 1
        sync()
        if multi:
            dist.barrier()
        reducer = getattr(tr, "reducer", None)
        if reducer is not None:
            reducer.exposed_ms(clear=True)  # drop the warm-up steps (the first one has no overlap)
        prof = None
        if args.profile and tr.info.rank == 0:
            from torch.profiler import ProfilerActivity, profile, schedule, tensorboard_trace_handler
            active = max(1, args.steps - 2)
            prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                           schedule=schedule(wait=1 if args.steps > 2 else 0, warmup=1 if args.steps > 1 else 0,
                                             active=active, repeat=1),
                           on_trace_ready=tensorboard_trace_handler("./bench_log"), record_shapes=True,
                           profile_memory=False, with_stack=False)
            prof.start()
        clk_before = None
        if cuda:
            from nanosandbox_amd.utils.boxcal import read_clocks
            clk_before = read_clocks(torch.device(tr.device).index or 0)
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss, _, X, Y = tr.train_step(X, Y)
            if prof is not None:
                prof.step()
        sync()
        if multi:
            dist.barrier()
        sync()
        dt = time.perf_counter() - t0
        dt_t = torch.tensor([dt], device=tr.device, dtype=torch.float64)
        if multi:
            dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
        dt = float(dt_t.item())
        exposed, early = None, None
        if reducer is not None:
            early = list(reducer.launched_in_backward)
            exposed = reducer.exposed_ms(clear=True)
            ex_t = torch.tensor(exposed or [0.0], device=tr.device, dtype=torch.float64)
            if multi:
                dist.all_reduce(ex_t, op=dist.ReduceOp.MAX)
            exposed = [float(v) for v in ex_t.tolist()] if exposed else []
        lossf = float(loss.item()) * tr.gas
        if prof is not None:
            prof.stop()
            print("profiler trace written under ./bench_log (not a clean timing: profiled steps)")
        box = None
        if cuda:
            # outside the timed region: DPM clock levels after the loop, then the calibration GEMM
            # (the same binary and shape on every box: its TF/s tells a slow box from slow code)
            clk_after = read_clocks(torch.device(tr.device).index or 0)
            cal = None
            if args.calib_seconds > 0:
                from nanosandbox_amd.utils.boxcal import calibration_gemm
                del X, Y
                cal = calibration_gemm(args.calib_seconds, tr.device)
            box = {"clocks_before": clk_before, "clocks_after": clk_after, "calibration": cal}
            if multi:
                every = [None] * world
                dist.all_gather_object(every, box)
                box = {"rank0": every[0], "calibration_tflops_by_rank": [
                    (b["calibration"] or {}).get("tflops") for b in every]}
            print(f"box: {json.dumps(box)}")

    tokens_per_step = tokens_per_micro * tr.gas * world
    value = tokens_per_step * args.steps / dt
    if emu:
        # one rank's share of the N-GPU step, measured; the job's rate is N x that share per step
        # time (every rank runs the same schedule), the collectives' time being the model's
        proj = {"projection": True, "per_rank_of": emu, "per_rank_ms": round(dt / args.steps * 1000.0, 3),
                "per_rank_tokens_per_step": tokens_per_step,
                "projected_tokens_per_s": round(emu * tokens_per_step * args.steps / dt, 1),
                "projected_global_batch": tokens_per_step * emu // args.block_size,
                "allreduce_model": tr.reducer.model(),
                "exposed_allreduce_ms": round(sum(exposed) / len(exposed), 3) if exposed else None,
                "buckets_launched_in_backward": list(early or [])}
        print(f"per-rank-of {emu} (PROJECTION): {json.dumps(proj)}", file=sys.stderr)
    ms = dt / args.steps * 1000.0
    flops_per_token = tr.raw_model.flops_per_token(args.block_size)
    mfu = value * flops_per_token / (world * 2.5e15)
    if tr.info.rank == 0:
        # nanoGPT bench.py's summary line (stderr; stdout carries only the JSON record)
        print(f"time per iteration: {ms:.4f}ms, MFU: {mfu * 100:.2f}%", file=sys.stderr)
        if emu:
            # a different record: the projected N-GPU rate, never the headline metric
            print(json.dumps({
                "metric": f"PROJECTED tokens/sec ({emu} GPUs) {args.model} DDP from one rank's share on 1 GPU",
                "value": proj["projected_tokens_per_s"], "unit": "tokens/s", "n_gpus": 1, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": proj["per_rank_ms"], "higher_is_better": True,
                "scaling": "strong", "vs_baseline": None, "dtype": "bf16" if args.dtype == "bfloat16" else "fp16",
                "data": "synthetic (uniform random tokens, vocab 50304); random-init weights",
                "config": {"model": args.model, "micro_batch": args.micro_batch, "grad_accum_per_rank": tr.gas,
                           "seq_len": args.block_size, "parallelism": f"dp{emu} (emulated, one rank)",
                           "bucket_mb": args.bucket_mb},
                "projection": proj, "box": box}), flush=True)
        else:
            print(json.dumps({
                "metric": METRIC if args.model == "gpt2" else f"tokens/sec (whole node) {args.model} DDP",
                "value": round(value, 1),
                "unit": "tokens/s",
                "n_gpus": world,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": round(ms, 3),
                "higher_is_better": True,
                "scaling": "strong",
                "vs_baseline": None,
                "dtype": ({"bfloat16": "bf16", "float16": "fp16"}[args.dtype]) if cuda else "fp32",
                "data": (f"real ({dataset}); random-init weights" if args.real_data else
                         "synthetic (uniform random tokens, vocab 50304); random-init weights"),
                "config": {"model": "GPT-2 124M" if args.model == "gpt2" else args.model,
                           "global_batch": tokens_per_step // args.block_size, "seq_len": args.block_size,
                           "tokens_per_step": tokens_per_step, "micro_batch": args.micro_batch,
                           "grad_accum_per_rank": tr.gas, "parallelism": f"dp{world}",
                           "ddp_impl": args.ddp_impl, "bucket_mb": args.bucket_mb,
                           "residual_dtype": "bf16" if args.bf16_residual else "fp32",
                           "deterministic": args.deterministic, "grad_ckpt": bool(tr.raw_model.grad_ckpt),
                       "recompute_mlp": bool(tr.raw_model.recompute_mlp),
                           "bias": args.bias},
                "peak_hbm_gib": round(torch.cuda.max_memory_allocated(tr.device) / 2 ** 30, 1) if cuda else None,
                "mfu_vs_2.5PF": round(mfu, 4),
                "loss": round(lossf, 4),
                # every GEMM shape of the step and the kernel that ran it (fixed rule,
                # ops/gemm_dispatch.py): a vendor-library pick would read "torch"
                "gemm_kernels": gemm_kernels,
                # N > 1: RCCL's transport per rank (from its INIT log) + the 64 MiB all-reduce, and
                # the bus bandwidth by message size (docs/rccl.md bucket sizing)
                "rccl": rccl_summary(getattr(tr, "rccl_report", None), sweep, reducer, exposed, early),
                # box calibration (not timed): DPM clock levels around the timed loop and a fixed
                # calibration GEMM's TF/s, so a slow box can be told from a regression
                "box": box,
            }), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
