"""HBM planning for a training micro-step: activation-memory estimate and the
grad-checkpointing decision.

nanoGPT leaves activation checkpointing to the user; on a 288 GB MI355X the question
is different: at nanoGPT's micro-batch 12 every GPT-2 size, 1.5B included, keeps all
of its activations resident with room to spare, and recomputing each block in the
backward (``grad_ckpt``) costs a third of the forward for nothing (GPT-2 1.5B, 60 x
1024 tokens per micro-step: 5043 ms/step resident vs 6750 ms checkpointed,
BASELINE.md).  ``plan_grad_ckpt`` therefore turns checkpointing on only when the
estimate below does not fit in the memory left after parameters, gradients and
optimizer state are allocated (config key ``hbm_plan``, on by default).

Per token, per layer, what the fused training path keeps for the backward
(fp32 residual stream, bf16 branch tensors; ``models/gpt.py`` + ``ops/functional.py``):

  ln_1 / ln_2 inputs (residual stream)   2 x 4C   (fp32; 2C each with a bf16 stream)
  ln_1 / ln_2 outputs                    2 x 2C   (weight-grad operands)
  packed qkv                             6C       (attention backward)
  attention output                       2C       (O for the backward, c_proj operand)
  c_fc output (pre-GELU)                 8C
  GELU output                            8C       (mlp.c_proj weight-grad operand)
  LSE + LayerNorm statistics             4H + 16

plus the bf16 logits / loss-gradient buffer(s) of the LM head (2V bytes each) and a
transient of roughly one layer's activations again during its backward.  With
checkpointing each block keeps only its input (fp32 x + bf16 ln output: 6C) and one
block at a time is recomputed.  ``calibration`` scales the estimate.

Measured on MI355X (``bench.py`` ``peak_hbm_gib`` = ``torch.cuda.max_memory_allocated``,
minus ~20 bytes/parameter of model state): the estimate is conservative by 4-29 %
(124M at 120 x 1024 tokens: 64.8 GiB estimated vs ~51 GiB; 350M: 129 vs ~114; 1.5B at
60 x 1024: 174 vs ~167; 1.5B checkpointed at 120 x 1024: 90 vs ~70).
"""

from __future__ import annotations

from dataclasses import dataclass

GiB = 1 << 30


@dataclass
class ActivationPlan:
    tokens: int
    resident_bytes: int      # activations with every block resident
    ckpt_bytes: int          # activations with per-block checkpointing
    budget_bytes: int        # memory available for activations (0 = unknown)
    grad_ckpt: bool          # the decision
    reason: str
    recompute_mlp: bool = False  # selective recomputation of the MLPs (between the two)
    mlp_recompute_bytes: int = 0

    def describe(self) -> str:
        return (f"activation plan: {self.tokens} tokens/micro-step, resident {self.resident_bytes / GiB:.1f} GiB, "
                f"MLP-recompute {self.mlp_recompute_bytes / GiB:.1f} GiB, checkpointed {self.ckpt_bytes / GiB:.1f} "
                f"GiB, budget {self.budget_bytes / GiB:.1f} GiB -> grad_ckpt={self.grad_ckpt} "
                f"recompute_mlp={self.recompute_mlp} ({self.reason})")


def layer_bytes_per_token(n_embd: int, n_head: int, fp32_residual: bool = True, recompute_mlp: bool = False) -> int:
    """Bytes one transformer block keeps per token for its backward (see module doc); with
    ``recompute_mlp`` the MLP keeps only its input (the c_fc output and GELU output, 16C, are
    recomputed in the backward: ops.functional.MLPFn)."""
    C = n_embd
    resid = 4 if fp32_residual else 2
    mlp = 0 if recompute_mlp else 8 * C + 8 * C
    return 2 * resid * C + 2 * 2 * C + 6 * C + 2 * C + mlp + 4 * n_head + 16


def activation_bytes(n_layer: int, n_embd: int, n_head: int, vocab_size: int, tokens: int,
                     fp32_residual: bool = True, grad_ckpt: bool = False, calibration: float = 1.0,
                     recompute_mlp: bool = False) -> int:
    """Estimated peak activation memory (bytes) of one forward + backward micro-step."""
    per_layer = layer_bytes_per_token(n_embd, n_head, fp32_residual, recompute_mlp and not grad_ckpt)
    resid = 4 if fp32_residual else 2
    head = 2 * 2 * vocab_size + (resid + 2) * n_embd  # logits + loss-gradient buffers, ln_f in/out
    if grad_ckpt:
        body = n_layer * (resid + 2) * n_embd + 2 * per_layer  # block inputs + one recomputed block (+ its grads)
    else:
        body = n_layer * per_layer + per_layer                   # all blocks + one block's gradient transient
    return int(calibration * tokens * (body + head))


def plan_grad_ckpt(n_layer: int, n_embd: int, n_head: int, vocab_size: int, tokens: int, free_bytes: int,
                   fp32_residual: bool = True, requested: bool = False, headroom: float = 0.9,
                   calibration: float = 1.0, recompute_mlp: bool = False) -> ActivationPlan:
    """Resident if it fits ``headroom`` x the free memory; else selective recomputation of the
    MLPs (one extra c_fc GEMM per layer) if that fits; else per-block checkpointing (a whole
    extra forward).

    ``requested`` (config ``grad_ckpt=True``) and ``recompute_mlp`` (config key of the same
    name) are always honoured; ``free_bytes`` = 0 means unknown (CPU runs): no automatic
    change."""
    kw = dict(n_layer=n_layer, n_embd=n_embd, n_head=n_head, vocab_size=vocab_size, tokens=tokens,
              fp32_residual=fp32_residual, calibration=calibration)
    res = activation_bytes(grad_ckpt=False, **kw)
    sel = activation_bytes(grad_ckpt=False, recompute_mlp=True, **kw)
    ck = activation_bytes(grad_ckpt=True, **kw)
    budget = int(headroom * free_bytes)

    def plan(gc, rm, why):
        return ActivationPlan(tokens, res, ck, budget, gc, why, recompute_mlp=rm, mlp_recompute_bytes=sel)
    if requested:
        return plan(True, False, "requested by config")
    if recompute_mlp:
        return plan(False, True, "MLP recompute requested by config")
    if free_bytes <= 0:
        return plan(False, False, "free memory unknown")
    if res <= budget:
        return plan(False, False, "fits resident")
    if sel <= budget:
        return plan(False, True, "resident estimate exceeds the budget; MLP recompute fits")
    return plan(True, False, "resident and MLP-recompute estimates exceed the budget" +
                ("" if ck <= budget else "; checkpointed may not fit either"))


def model_state_bytes(n_layer: int, n_embd: int, vocab_size: int, block_size: int) -> int:
    """Parameters, gradients and optimizer state of a GPT-2-shaped model: fp32 master
    weights + fp32 flat gradient + two fp32 Adam moments + the bf16 compute copy and its
    cached transposes (~20 bytes per parameter)."""
    n_params = 12 * n_layer * n_embd * n_embd + (vocab_size + block_size) * n_embd
    return 20 * n_params


RUNTIME_RESERVE = 8 * GiB  # HIP context, library workspaces, allocator slack: the trainer's
# free-memory reading after model setup sits ~4 GiB below total - model state


def choose_micro_batch(n_layer: int, n_embd: int, n_head: int, vocab_size: int, block_size: int,
                       per_rank_seqs: int, hbm_bytes: int, fp32_residual: bool = True, cap: int = 120,
                       headroom: float = 0.9) -> tuple[int, bool]:
    """(micro-batch, grad_ckpt) for a rank that must process ``per_rank_seqs`` sequences per
    optimizer step: the largest divisor of per_rank_seqs (<= cap) whose activations stay
    resident in ``hbm_bytes`` next to the model state; if even a one-sequence micro-step
    would not fit, the largest divisor whose checkpointed activations fit, with grad_ckpt.
    Larger micro-steps amortise the per-launch costs; resident beats checkpointed at any
    micro-batch (GPT-2 1.5B: 60 resident 4592 ms/step in round 3, 120 checkpointed 6779 in round 2)."""
    budget = headroom * (hbm_bytes - model_state_bytes(n_layer, n_embd, vocab_size, block_size) - RUNTIME_RESERVE)
    divisors = [d for d in range(min(cap, per_rank_seqs), 0, -1) if per_rank_seqs % d == 0]
    kw = dict(n_layer=n_layer, n_embd=n_embd, n_head=n_head, vocab_size=vocab_size, fp32_residual=fp32_residual)
    for d in divisors:
        if activation_bytes(tokens=d * block_size, **kw) <= budget:
            return d, False
    for d in divisors:
        if activation_bytes(tokens=d * block_size, grad_ckpt=True, **kw) <= budget:
            return d, True
    return divisors[-1], True
