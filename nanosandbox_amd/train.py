"""Trainer: nanoGPT's ``train.py`` contract on the MI355X-native stack.

Usage (identical CLI to nanoGPT; reference
``notebooks/colab_nanoGPT_companion.ipynb:70-79,107-116``)::

    python train.py config/train_shakespeare_char.py --device=cpu --compile=False
    torchrun --standalone --nproc_per_node=8 train.py config/train_gpt2.py --dataset=synthetic

What is the same: config keys and defaults, distributed init, grad accumulation
(divided by world size), cosine LR, eval/checkpoint cadence and rules, resume,
stdout log lines, checkpoint layout.

What is MI355X-native: parameters/grads/optimizer state in flat HBM buffers,
bf16 compute weights maintained by the fused AdamW kernel, HIP kernels for
every non-GEMM op, our bucketed RCCL reducer instead of torch DDP (``ddp_impl``
keeps torch DDP selectable), evaluation through the unwrapped module (avoids
the reference's DDP-forward-on-rank-0 hazard), JSONL +
tfevents metrics, atomic checkpoints, opt-in auto-resume and fault injection
for elastic restarts.
"""

from __future__ import annotations

import os
import sys
import time

import torch

from .config import TRAIN_DEFAULTS, config_keys, parse_argv
from .data import load_meta, make_batch_source, resolve_data_dir
from .ops import rng_advance
from .ops.functional import XENT_F16_GUARD as xent_f16_guard
from .runtime import MicroStepGraph, graph_capture_supported
from .models import GPT, GPTConfig
from .optim import FlatParamStore
from .parallel import FlatBucketReducer, destroy, init_distributed
from .utils import MetricsLogger, get_lr, load_checkpoint, load_model_state, save_checkpoint


_DTYPES = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32}


def _compute_dtype(device_type: str, dtype: str) -> torch.dtype:
    """nanoGPT's ``dtype`` key: 'bfloat16' (default on MI355X), 'float16' (with a dynamic loss
    scale) or 'float32'.  On the GPU bf16 and fp16 run our HIP kernels (the
    fp16 ones are the same sources with v_mfma_*_f16 and fp16 conversions; gfx950's fp16 MFMA
    rate equals bf16's); fp32 runs every op's torch reference implementation (the numerics
    contract, at library speed).  The CPU always computes in fp32 (nanoGPT: nullcontext on
    CPU)."""
    if dtype not in _DTYPES:
        raise ValueError(f"dtype must be one of {sorted(_DTYPES)}, got {dtype!r}")
    if device_type != "cuda":
        return torch.float32
    return _DTYPES[dtype]


class Trainer:
    def __init__(self, cfg: dict):
        self.cfg = cfg
        c = cfg
        self.info = init_distributed(c["backend"], c["device"])
        info = self.info
        self.device = info.device
        self.device_type = "cuda" if "cuda" in self.device else "cpu"
        self.master = info.master_process
        if info.ddp and os.environ.get("NSA_LOCAL_DEVICE", "").strip():
            # Topology B over xGMI: the launcher picked this pod's GPU by its ordinal
            print(f"rank {info.rank}: device by ordinal NSA_LOCAL_DEVICE={os.environ['NSA_LOCAL_DEVICE']} -> "
                  f"{self.device}", flush=True)
        gas = c["gradient_accumulation_steps"]
        if info.ddp:
            assert gas % info.world_size == 0
            gas //= info.world_size
        self.gas = gas
        self.tokens_per_iter = gas * info.world_size * c["batch_size"] * c["block_size"]
        if self.master:
            print(f"tokens per iteration will be: {self.tokens_per_iter:,}")
            os.makedirs(c["out_dir"], exist_ok=True)
        torch.manual_seed(c["seed"] + info.seed_offset)
        self.compute_dtype = _compute_dtype(self.device_type, c["dtype"])
        # nanoGPT: GradScaler(enabled=(dtype == 'float16')) -- a no-op off the GPU
        self.scaler = None
        if self.compute_dtype == torch.float16:
            from .optim.loss_scale import DynamicLossScale
            self.scaler = DynamicLossScale(device=self.device)
        if self.device_type == "cuda" and self.compute_dtype != torch.bfloat16 and self.master:
            print(f"dtype={c['dtype']}: " + ("fp16 HIP kernels, dynamic loss scale on the device" if self.scaler
                                            else "torch reference ops (the HIP kernels run bf16 / fp16)"))

        # ---------------------------------------------------------------- data
        self.data_dir = resolve_data_dir(c["dataset"], c["data_dir"])
        meta = load_meta(self.data_dir) if c["dataset"] != "synthetic" else None
        meta_vocab_size = meta["vocab_size"] if meta else None
        if meta_vocab_size is not None:
            print(f"found vocab_size = {meta_vocab_size} (inside {self.data_dir})")

        # --------------------------------------------------------------- model
        init_from = c["init_from"]
        ckpt_path = os.path.join(c["out_dir"], "ckpt.pt")
        if c["auto_resume"] and os.path.exists(ckpt_path):
            print(f"auto_resume: found {ckpt_path}")
            init_from = "resume"
        model_args = dict(n_layer=c["n_layer"], n_head=c["n_head"], n_embd=c["n_embd"], block_size=c["block_size"],
                          bias=c["bias"], vocab_size=None, dropout=c["dropout"])
        self.iter_num = 0
        self.best_val_loss = 1e9
        checkpoint = None
        if init_from == "scratch":
            print("Initializing a new model from scratch")
            if meta_vocab_size is None:
                print("defaulting to vocab_size of GPT-2 to 50304 (50257 rounded up for efficiency)")
            model_args["vocab_size"] = meta_vocab_size if meta_vocab_size is not None else 50304
            model = GPT(GPTConfig(**model_args))
        elif init_from == "resume":
            print(f"Resuming training from {c['out_dir']}")
            checkpoint = load_checkpoint(ckpt_path, map_location="cpu")
            for k in ["n_layer", "n_head", "n_embd", "block_size", "bias", "vocab_size"]:
                model_args[k] = checkpoint["model_args"][k]
            model = GPT(GPTConfig(**model_args))
            load_model_state(model, checkpoint["model"])
            self.iter_num = checkpoint["iter_num"]
            self.best_val_loss = float(checkpoint["best_val_loss"])
        elif init_from.startswith("gpt2"):
            print(f"Initializing from OpenAI GPT-2 weights: {init_from}")
            model = GPT.from_pretrained(init_from, dict(dropout=c["dropout"]))
            for k in ["n_layer", "n_head", "n_embd", "block_size", "bias", "vocab_size"]:
                model_args[k] = getattr(model.config, k)
        else:
            raise ValueError(f"unknown init_from {init_from!r}")
        if c["block_size"] < model.config.block_size:
            model.crop_block_size(c["block_size"])
            model_args["block_size"] = c["block_size"]
        self.model_args = model_args
        model.to(self.device)
        model.set_compute_dtype(self.compute_dtype,
                                torch.float32 if c["fp32_residual"] else self.compute_dtype)
        model.grad_ckpt = c["grad_ckpt"]
        model.recompute_mlp = c["recompute_mlp"]
        from . import ops as _ops
        _ops.set_deterministic(c["deterministic"])
        # the dropout kernels' device step counter: a fresh run starts its stream at 0, a
        # resumed one continues where the checkpointed run stood (micro-steps taken so far)
        # instead of replaying the first steps' masks
        _ops.rng_set(self.device, self.iter_num * self.gas)
        print(f"number of parameters: {model.get_num_params() / 1e6:.2f}M")

        # ------------------------------------------- flat store + fused AdamW
        self.ddp_impl = c["ddp_impl"] if info.ddp else "none"
        fused_grad = self.ddp_impl != "torch"
        # the 16-bit compute shadow the fused AdamW kernel rewrites each step (bf16 or fp16)
        shadow = self.compute_dtype if self.compute_dtype in (torch.bfloat16, torch.float16) else None
        self.store = FlatParamStore(model, self.device, compute_dtype=shadow if self.device_type == "cuda" else None,
                                    fused_grad=fused_grad)
        self.optimizer = model.configure_optimizers(c["weight_decay"], c["learning_rate"], (c["beta1"], c["beta2"]),
                                                    self.device_type, store=self.store)
        if self.scaler is not None:
            self.optimizer.attach_loss_scale(self.scaler)  # inf check / skip / update on the device
        if init_from == "resume" and checkpoint is not None:
            self.optimizer.load_state_dict(checkpoint["optimizer"])
        checkpoint = None  # free up memory
        # HBM plan (utils/memory.py): with parameters, gradients and optimizer state now
        # allocated, keep every block's activations resident unless they do not fit
        self.activation_plan = None
        if self.device_type == "cuda" and (c["grad_ckpt"] or c["hbm_plan"]):
            from .utils.memory import plan_grad_ckpt
            free, _ = torch.cuda.mem_get_info(torch.device(self.device))
            self.activation_plan = plan_grad_ckpt(
                model.config.n_layer, model.config.n_embd, model.config.n_head, model.config.vocab_size,
                c["batch_size"] * c["block_size"], free, fp32_residual=c["fp32_residual"], requested=c["grad_ckpt"],
                recompute_mlp=c["recompute_mlp"])
            model.grad_ckpt = self.activation_plan.grad_ckpt
            model.recompute_mlp = self.activation_plan.recompute_mlp
            if self.master:
                print(self.activation_plan.describe())
        # compile=True: no Triton/Inductor on this stack; the micro-step (forward +
        # backward) is captured once as a HIP graph and replayed (runtime/hipgraph.py)
        self.graph = None
        self.use_graph = False
        if c["compile"]:
            ok, why = graph_capture_supported(self.device, c["dropout"], info.world_size, self.ddp_impl, self.gas)
            if ok and self.compute_dtype not in (torch.bfloat16, torch.float16):
                ok, why = False, f"dtype={c['dtype']} runs the torch reference ops"
            self.use_graph = ok
            if self.master:
                print(("compile=True: micro-step captured as a HIP graph" +
                       (" (the synchronising micro-step runs eagerly)" if info.world_size > 1 else "")) if ok
                      else f"compile=True: eager micro-steps ({why})")

        # ----------------------------------------------------------------- DDP
        self.raw_model = model
        self.model = model
        self.reducer = None
        if info.ddp:
            if self.ddp_impl == "flat":
                rdt = torch.bfloat16 if c["grad_reduce_dtype"] == "bfloat16" else torch.float32
                self.reducer = FlatBucketReducer(self.store, bucket_cap_mb=c["ddp_bucket_mb"], reduce_dtype=rdt)
                self.reducer.broadcast_parameters()
                self.optimizer.grad_scale = self.reducer.grad_scale
                if self.master:
                    print(f"DDP: flat bucketed reducer, {len(self.reducer.buckets)} buckets "
                          f"(cap {c['ddp_bucket_mb']} MiB, {c['grad_reduce_dtype']})")
            elif self.ddp_impl == "torch":
                from torch.nn.parallel import DistributedDataParallel as DDP
                dev_ids = [torch.device(self.device).index] if self.device_type == "cuda" else None
                self.model = DDP(model, device_ids=dev_ids, bucket_cap_mb=c["ddp_bucket_mb"])
                self.store.refresh_compute()
            else:
                raise ValueError(f"unknown ddp_impl {self.ddp_impl!r}")

        if info.ddp and c["rccl_report"]:
            # which transport RCCL picked per peer (P2P over xGMI / SHM / NET) and the bus
            # bandwidth of one 64 MiB all-reduce (docs/rccl.md)
            from .parallel import report_transport
            self.rccl_report = report_transport(info)

        self._grad_scale0 = self.optimizer.grad_scale  # 1/world (flat reducer) or 1
        self.batches = make_batch_source(c["dataset"], c["data_dir"], c["block_size"], c["batch_size"], self.device,
                                         seed=c["seed"] + info.seed_offset, vocab_size=model_args["vocab_size"])
        run_name = c["wandb_run_name"] or "run"
        self.metrics = MetricsLogger(c["out_dir"], jsonl=c["metrics_jsonl"], tensorboard_dir=c["tensorboard_dir"],
                                     run_name=run_name, enabled=self.master)
        if c["wandb_log"] and self.master:
            print("wandb_log=True: wandb is not installed in this image; logging to metrics.jsonl/tfevents instead")

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def estimate_loss(self):
        out = {}
        m = self.raw_model  # never forward the DDP wrapper on one rank (SURVEY.md §2.8 hazard)
        m.eval()
        for split in ["train", "val"]:
            losses = torch.zeros(self.cfg["eval_iters"], device=self.device)
            for k in range(self.cfg["eval_iters"]):
                X, Y = self.batches.get_batch(split)
                _, loss = m(X, Y)
                losses[k] = loss.float()
            out[split] = losses.mean().item()
        m.train()
        return out

    def _save(self):
        print(f"saving checkpoint to {self.cfg['out_dir']}")
        save_checkpoint(os.path.join(self.cfg["out_dir"], "ckpt.pt"), self.raw_model, self.optimizer,
                        self.model_args, self.iter_num, self.best_val_loss,
                        {k: self.cfg[k] for k in config_keys(self.cfg)})

    # ------------------------------------------------------------------ step
    def train_step(self, X, Y):
        """One optimizer iteration (grad_accum micro-steps + clip + fused AdamW).

        Returns (last micro-step loss tensor, grad-norm tensor or None, next X, next Y)."""
        c = self.cfg
        # with a reducer (world > 1) the synchronising last micro-step runs eagerly below
        n_graph = (self.gas - 1 if self.reducer is not None else self.gas) if self.use_graph else 0
        if n_graph > 0:
            if self.graph is None:
                if self.reducer is not None:
                    self.reducer.prepare(False)  # capture with the bucket hooks disarmed
                self.graph = MicroStepGraph(self.model, X, Y, self.gas,
                                            zero_grad=lambda: self.optimizer.zero_grad(set_to_none=True),
                                            dropout=c["dropout"] > 0.0,
                                            loss_scale=self.scaler.scale_t if self.scaler is not None else None)
            for _ in range(n_graph):
                loss = self.graph.run(X, Y)
                X, Y = self.batches.get_batch("train")
        for micro_step in range(n_graph, self.gas):
            sync = micro_step == self.gas - 1
            if self.reducer is not None:
                self.reducer.prepare(sync)
            elif self.ddp_impl == "torch":
                self.model.require_backward_grad_sync = sync
            if c["dropout"] > 0.0:
                rng_advance(self.device)  # the dropout kernels' device step counter (graph-safe RNG)
            _, loss = self.model(X, Y)
            loss = loss / self.gas  # scale the loss to account for gradient accumulation
            # immediately async prefetch next batch while model is doing the forward pass on the GPU
            X, Y = self.batches.get_batch("train")
            # fp16: the loss times the device-resident scale (no host sync); the optimizer's
            # kernels unscale, check for inf / NaN, skip and update the scale (loss_scale.py)
            (loss * self.scaler.scale_t if self.scaler is not None else loss).backward()
        if self.reducer is not None:
            self.reducer.finish()
        norm = None
        if c["grad_clip"] != 0.0:
            norm = self.optimizer.clip_grad_norm_(c["grad_clip"])
        self.optimizer.step()
        if norm is None and self.scaler is not None and hasattr(self.optimizer, "last_norm"):
            norm = self.optimizer.last_norm  # fp16 without clipping: the step's own inf check (inf = skipped)
        self.optimizer.zero_grad(set_to_none=True)
        if self.scaler is not None and xent_f16_guard.poll():
            self.graph = None  # captured with the fused fp16 cross-entropy: recapture on the next step
        return loss, norm, X, Y

    def fit(self):
        c = self.cfg
        X, Y = self.batches.get_batch("train")
        t0 = time.time()
        local_iter_num = 0
        running_mfu = -1.0
        prof = self._profiler() if c["profile"] and self.master else None
        while True:
            lr = get_lr(self.iter_num, c["learning_rate"], c["warmup_iters"], c["lr_decay_iters"], c["min_lr"]) \
                if c["decay_lr"] else c["learning_rate"]
            for param_group in self.optimizer.param_groups:
                param_group["lr"] = lr

            if self.iter_num % c["eval_interval"] == 0 and self.master:
                losses = self.estimate_loss()
                print(f"step {self.iter_num}: train loss {losses['train']:.4f}, val loss {losses['val']:.4f}")
                self.metrics.log("eval", self.iter_num, train_loss=losses["train"], val_loss=losses["val"], lr=lr)
                if losses["val"] < self.best_val_loss or c["always_save_checkpoint"]:
                    self.best_val_loss = losses["val"]
                    if self.iter_num > 0:
                        self._save()
            if self.iter_num == 0 and c["eval_only"]:
                break
            if c["fault_inject_iter"] == self.iter_num and c["fault_inject_rank"] == self.info.rank:
                self._inject_fault()

            loss, norm, X, Y = self.train_step(X, Y)
            if prof is not None:
                prof.step()

            t1 = time.time()
            dt = t1 - t0
            t0 = t1
            if self.iter_num % c["log_interval"] == 0 and self.master:
                lossf = loss.item() * self.gas
                if local_iter_num >= 5:  # let the training loop settle a bit
                    mfu = self.raw_model.estimate_mfu(c["batch_size"] * self.gas, dt)  # per-GPU, as nanoGPT
                    running_mfu = mfu if running_mfu == -1.0 else 0.9 * running_mfu + 0.1 * mfu
                print(f"iter {self.iter_num}: loss {lossf:.4f}, time {dt * 1000:.2f}ms, mfu {running_mfu * 100:.2f}%")
                extra = {"grad_norm": float(norm.item())} if norm is not None else {}
                self.metrics.log("train", self.iter_num, loss=lossf, lr=lr, dt_ms=dt * 1000,
                                 tokens_per_s=self.tokens_per_iter / dt, mfu=running_mfu, **extra)
            self.iter_num += 1
            local_iter_num += 1
            if self.iter_num > c["max_iters"]:
                break
        if prof is not None:
            prof.stop()
        self.metrics.close()
        if os.environ.get("NSA_PARAM_DIGEST") == "1":
            # replica-consistency probe for the elastic-restart test: every rank prints a
            # digest of its parameters; DDP replicas must agree bit for bit
            import hashlib
            h = hashlib.sha256()
            for _, p in sorted(self.raw_model.state_dict().items()):
                h.update(p.detach().float().cpu().numpy().tobytes())
            print(f"param digest rank {self.info.rank}: {h.hexdigest()[:16]} iter {self.iter_num}", flush=True)

    def _inject_fault(self):
        """Fail this rank once per job (SURVEY.md §5.3 fault injection).

        The fault fires only on the job's first attempt: a marker file in ``out_dir``
        (shared storage: the PVC in the k8s topologies) records that it fired, and
        torchrun's ``TORCHELASTIC_RESTART_COUNT`` > 0 also suppresses it, so an elastic
        restart (``--max-restarts``) that auto-resumes from ``ckpt.pt`` runs through.  The
        marker is keyed to the job, so a later job reusing the same out_dir still gets its
        fault: torchrun's ``TORCHELASTIC_RUN_ID`` when it names the job; under torchrun's
        default ``--rdzv-id`` ("none", shared by every default launch) the elastic agent's pid
        (the workers' parent, unchanged across that job's restarts); else this process."""
        job = _fault_job_key()
        job = "".join(ch if ch.isalnum() or ch in "-_" else "_" for ch in job)
        marker = os.path.join(self.cfg["out_dir"], f".fault_injected_rank{self.info.rank}.{job}")
        if os.path.exists(marker) or int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") or 0) > 0:
            return
        os.makedirs(self.cfg["out_dir"], exist_ok=True)
        with open(marker, "w") as f:
            f.write(f"{self.iter_num}\n")
        raise RuntimeError(f"injected fault at iter {self.iter_num} on rank {self.info.rank}")

    def _profiler(self):
        from torch.profiler import ProfilerActivity, profile, schedule, tensorboard_trace_handler
        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if self.device_type == "cuda" else [])
        p = profile(activities=acts, schedule=schedule(wait=5, warmup=5, active=5, repeat=1),
                    on_trace_ready=tensorboard_trace_handler(os.path.join(self.cfg["out_dir"], "trace")),
                    record_shapes=True, profile_memory=True)
        p.start()
        return p


def _fault_job_key() -> str:
    """Job identity for the fault-injection marker (see ``Trainer._inject_fault``)."""
    run_id = os.environ.get("TORCHELASTIC_RUN_ID", "")
    if run_id and run_id.lower() != "none":
        return f"run{run_id}"
    if "TORCHELASTIC_RESTART_COUNT" in os.environ:  # under torchrun with the default rdzv id
        return f"agent{os.getppid()}"
    return f"pid{os.getpid()}"


def main(argv=None):
    cfg = parse_argv(TRAIN_DEFAULTS, sys.argv[1:] if argv is None else argv)
    trainer = Trainer(cfg)
    try:
        trainer.fit()
    finally:
        destroy()
    return trainer


if __name__ == "__main__":
    main()
