"""GPT-2 family model with nanoGPT's module names, init and API.

Behavioural contract: SURVEY.md §2.3 rows U-M1..U-M11 (upstream nanoGPT
``model.py``, executed by reference ``notebooks/colab_nanoGPT_companion.ipynb:39,70``).
State-dict keys, weight tying (``transformer.wte.weight is lm_head.weight``),
init (N(0, 0.02), zero biases, ``*c_proj.weight`` at 0.02/sqrt(2·n_layer)),
``configure_optimizers``/``estimate_mfu``/``generate``/``crop_block_size``/
``from_pretrained`` all follow that contract so nanoGPT checkpoints load.

What differs is the execution: ``nn.Linear``/``nn.Embedding`` are used only
as parameter containers; ``forward`` runs our fused ops
(``nanosandbox_amd.ops``): HIP LayerNorm / GELU / flash attention / embedding
/ fused lm_head+cross-entropy kernels on gfx950, residual adds folded into
the projection GEMMs, and weight gradients accumulated in fp32 straight into
the flat gradient buffer.
"""

from __future__ import annotations

import inspect
import math
from dataclasses import dataclass

import torch
import torch.nn as nn
from torch.utils.checkpoint import checkpoint

from .. import ops

# MI355X dense bf16 peak (MI355X_MICROARCH.md "Peak BF16/FP16 MFMA ~2.5 PF dense").
MI355X_BF16_PEAK_FLOPS = 2.5e15


@dataclass
class GPTConfig:
    block_size: int = 1024
    vocab_size: int = 50304  # GPT-2 vocab_size of 50257, padded up to nearest multiple of 64 for efficiency
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    dropout: float = 0.0
    bias: bool = True  # True: bias in Linears and LayerNorms, like GPT-2. False: a bit better and faster


class LayerNorm(nn.Module):
    """LayerNorm with an optional bias (PyTorch's lacks ``bias=False`` in old versions)."""

    def __init__(self, ndim, bias):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(ndim))
        self.bias = nn.Parameter(torch.zeros(ndim)) if bias else None
        self.out_dtype = None  # compute dtype of the normalised output (None: x's dtype)

    def forward(self, x):
        return ops.layer_norm(x, self.weight, self.bias, out_dtype=self.out_dtype)


class CausalSelfAttention(nn.Module):
    def __init__(self, config):
        super().__init__()
        assert config.n_embd % config.n_head == 0
        # key, query, value projections for all heads, packed: [q | k | v]
        self.c_attn = nn.Linear(config.n_embd, 3 * config.n_embd, bias=config.bias)
        # output projection
        self.c_proj = nn.Linear(config.n_embd, config.n_embd, bias=config.bias)
        self.n_head = config.n_head
        self.n_embd = config.n_embd
        self.dropout = config.dropout
        self.flash = True  # always: our flash kernel (gfx950) / fp32 reference on CPU

    def forward(self, x, resid_drop=True):
        """resid_dropout(c_proj(attn(c_attn(x)))) — the residual add is fused downstream
        (``resid_drop=False``: without the resid dropout, which the fused add + LayerNorm
        then applies)."""
        qkv = ops.linear(x, self.c_attn.weight, self.c_attn.bias)
        y = ops.attention(qkv, self.n_head, self.dropout, self.training)
        y = ops.linear(y, self.c_proj.weight, self.c_proj.bias)
        return ops.dropout(y, self.dropout, self.training) if resid_drop else y


class MLP(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.c_fc = nn.Linear(config.n_embd, 4 * config.n_embd, bias=config.bias)
        self.c_proj = nn.Linear(4 * config.n_embd, config.n_embd, bias=config.bias)
        self.dropout = config.dropout
        self.recompute = False  # selective recomputation (GPT.recompute_mlp)

    def forward(self, x, resid_drop=True):
        y = ops.mlp(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias,
                    recompute=self.recompute and self.training and torch.is_grad_enabled())
        return ops.dropout(y, self.dropout, self.training) if resid_drop else y


class Block(nn.Module):
    """Pre-norm block ``x = x + attn(ln_1(x)); x = x + mlp(ln_2(x))``.

    The hot path (``fused_forward``) takes ``h = ln_1(x)`` already computed and
    returns the MLP branch un-added: every residual add is fused with the
    LayerNorm that follows it (``ops.add_layer_norm``), so the residual stream
    is read/written once per add and the backward needs no gradient-sum kernel.
    """

    def __init__(self, config):
        super().__init__()
        self.ln_1 = LayerNorm(config.n_embd, bias=config.bias)
        self.attn = CausalSelfAttention(config)
        self.ln_2 = LayerNorm(config.n_embd, bias=config.bias)
        self.mlp = MLP(config)

    def resid_p(self):
        """nanoGPT's resid_dropout probability, applied by the fused add + LayerNorm."""
        return self.mlp.dropout if self.training else 0.0

    def fused_forward(self, x, h, split_grad=False):
        """(x + drop(attn(h)), mlp(ln_2(...))): the MLP branch returned un-added and without
        its resid dropout (the caller's add_layer_norm applies ``resid_p``)."""
        x, h2 = ops.add_layer_norm(x, self.attn(h, resid_drop=False), self.ln_2.weight, self.ln_2.bias,
                                   split_grad=split_grad, drop_p=self.resid_p())
        return x, self.mlp(h2, resid_drop=False)

    def forward(self, x):
        x, y = self.fused_forward(x, self.ln_1(x))
        return x + ops.dropout(y, self.mlp.dropout, self.training)


def _block_step(block, next_ln, x, h):
    # the trunk's residual stream runs from one fused LayerNorm to the next with no other
    # reader, so its gradient may travel split (ops.add_layer_norm split_grad)
    x, y = block.fused_forward(x, h, split_grad=True)
    return ops.add_layer_norm(x, y, next_ln.weight, next_ln.bias, split_grad=True, drop_p=block.resid_p())


class GPT(nn.Module):
    def __init__(self, config: GPTConfig):
        super().__init__()
        assert config.vocab_size is not None
        assert config.block_size is not None
        self.config = config
        self.grad_ckpt = False
        self.compute_dtype = torch.float32
        self.residual_dtype = torch.float32

        self.transformer = nn.ModuleDict(dict(
            wte=nn.Embedding(config.vocab_size, config.n_embd),
            wpe=nn.Embedding(config.block_size, config.n_embd),
            drop=nn.Dropout(config.dropout),
            h=nn.ModuleList([Block(config) for _ in range(config.n_layer)]),
            ln_f=LayerNorm(config.n_embd, bias=config.bias),
        ))
        self.lm_head = nn.Linear(config.n_embd, config.vocab_size, bias=False)
        # weight tying (https://paperswithcode.com/method/weight-tying)
        self.transformer.wte.weight = self.lm_head.weight
        # a vocabulary the lm_head GEMM kernel cannot tile exactly (GPT-2's 50257, a char
        # vocab of 65) runs on zero-padded rows: ask the flat store for the room
        pad = ops.lm_head_rows(config.vocab_size)
        if pad != config.vocab_size:
            self.lm_head.weight._nsa_pad_rows = pad
        # wte and wpe receive their last gradient contribution from the embedding backward,
        # the final kernel of the backward pass: the flat store gives them a tail bucket of
        # their own so no block weight waits behind them for its all-reduce
        self.transformer.wte.weight._nsa_late_grad = True
        self.transformer.wpe.weight._nsa_late_grad = True

        # init all weights
        self.apply(self._init_weights)
        # apply special scaled init to the residual projections, per GPT-2 paper
        for pn, p in self.named_parameters():
            if pn.endswith("c_proj.weight"):
                torch.nn.init.normal_(p, mean=0.0, std=0.02 / math.sqrt(2 * config.n_layer))

    # ------------------------------------------------------------------ utils
    def get_num_params(self, non_embedding=True):
        """Parameter count; position embeddings are subtracted by default (token
        embeddings stay, since they are tied to the lm_head)."""
        n_params = sum(p.numel() for p in self.parameters())
        if non_embedding:
            n_params -= self.transformer.wpe.weight.numel()
        return n_params

    def _init_weights(self, module):
        if isinstance(module, nn.Linear):
            torch.nn.init.normal_(module.weight, mean=0.0, std=0.02)
            if module.bias is not None:
                torch.nn.init.zeros_(module.bias)
        elif isinstance(module, nn.Embedding):
            torch.nn.init.normal_(module.weight, mean=0.0, std=0.02)

    @property
    def recompute_mlp(self) -> bool:
        """Selective recomputation: every MLP keeps only its input and recomputes its c_fc GEMM
        and GELU in the backward (~44 % of a block's resident activations, ~1 GEMM per layer of
        extra work), between fully resident blocks and per-block checkpointing (``grad_ckpt``)."""
        return bool(self.transformer.h) and self.transformer.h[0].mlp.recompute

    @recompute_mlp.setter
    def recompute_mlp(self, flag: bool):
        for block in self.transformer.h:
            block.mlp.recompute = bool(flag)

    def set_compute_dtype(self, dtype: torch.dtype, residual_dtype: torch.dtype = torch.float32):
        """Activation dtype of the forward pass (bf16 on MI355X, fp32 on CPU).

        ``residual_dtype`` is the dtype of the residual stream (embedding sum, the
        x of ``x = x + f(ln(x))``) and of its gradient.  fp32 by default: that is
        nanoGPT's autocast contract, where the embedding output is fp32 and every
        fp32 + bf16 residual add promotes to fp32.  bf16 halves the residual bytes
        (opt-in, ``fp32_residual=False``)."""
        self.compute_dtype = dtype
        # bf16 and fp16 (with the dynamic loss scale) compute run our kernels; fp32 compute takes
        # the torch reference path of every op (train.py --dtype); fp16 / fp32 keep an fp32
        # residual stream
        self.residual_dtype = residual_dtype if dtype == torch.bfloat16 else torch.float32
        for m in self.modules():
            if isinstance(m, LayerNorm):
                m.out_dtype = dtype
        return self

    # ---------------------------------------------------------------- forward
    def forward(self, idx, targets=None):
        b, t = idx.size()
        assert t <= self.config.block_size, \
            f"Cannot forward sequence of length {t}, block size is only {self.config.block_size}"
        tr = self.transformer
        x = ops.embedding(idx, tr.wte.weight, tr.wpe.weight, self.config.dropout, self.training,
                          dtype=self.residual_dtype, cdtype=self.compute_dtype)
        x = self._trunk(x)

        if targets is not None:
            loss = ops.lm_head_loss(x, self.lm_head.weight, targets)
            logits = None  # the [B,T,V] logits are consumed in place by the fused CE kernel
        else:
            # inference-time mini-optimization: only forward the lm_head on the very last position
            logits = ops.lm_head_logits(x[:, [-1], :], self.lm_head.weight)
            loss = None
        return logits, loss

    def _trunk(self, x):
        """Blocks + ln_f with every residual add fused into the following LayerNorm."""
        tr = self.transformer
        blocks = tr.h
        ln = blocks[0].ln_1
        x, h = ops.layer_norm_pass(x, ln.weight, ln.bias, out_dtype=ln.out_dtype)
        ckpt = self.grad_ckpt and self.training and torch.is_grad_enabled()
        for i, block in enumerate(blocks):
            nxt = blocks[i + 1].ln_1 if i + 1 < len(blocks) else tr.ln_f
            if ckpt:
                x, h = checkpoint(_block_step, block, nxt, x, h, use_reentrant=False)
            else:
                x, h = _block_step(block, nxt, x, h)
        return h

    def forward_logits(self, idx):
        """Full [B, T, V] fp32 logits (evaluation / tests)."""
        tr = self.transformer
        x = ops.embedding(idx, tr.wte.weight, tr.wpe.weight, 0.0, False, dtype=self.residual_dtype,
                          cdtype=self.compute_dtype)
        return ops.lm_head_logits(self._trunk(x), self.lm_head.weight)

    # ------------------------------------------------------------ surgery/api
    def crop_block_size(self, block_size):
        """Model surgery to decrease the block size if necessary (e.g. load gpt2 at 1024, use 256)."""
        assert block_size <= self.config.block_size
        self.config.block_size = block_size
        self.transformer.wpe.weight = nn.Parameter(self.transformer.wpe.weight[:block_size].detach().clone())
        for block in self.transformer.h:
            if hasattr(block.attn, "bias"):
                block.attn.bias = block.attn.bias[:, :, :block_size, :block_size]

    @classmethod
    def from_pretrained(cls, model_type, override_args=None):
        """Load OpenAI GPT-2 weights from a local HuggingFace snapshot (no network here)."""
        from ..utils.hf import load_hf_gpt2_state_dict
        assert model_type in {"gpt2", "gpt2-medium", "gpt2-large", "gpt2-xl"}
        override_args = override_args or {}
        assert all(k == "dropout" for k in override_args)
        config_args = {
            "gpt2": dict(n_layer=12, n_head=12, n_embd=768),  # 124M params
            "gpt2-medium": dict(n_layer=24, n_head=16, n_embd=1024),  # 350M params
            "gpt2-large": dict(n_layer=36, n_head=20, n_embd=1280),  # 774M params
            "gpt2-xl": dict(n_layer=48, n_head=25, n_embd=1600),  # 1558M params
        }[model_type]
        print(f"loading weights from pretrained gpt: {model_type}")
        config_args["vocab_size"] = 50257
        config_args["block_size"] = 1024
        config_args["bias"] = True
        if "dropout" in override_args:
            print(f"overriding dropout rate to {override_args['dropout']}")
            config_args["dropout"] = override_args["dropout"]
        model = GPT(GPTConfig(**config_args))
        sd = model.state_dict()
        sd_hf = load_hf_gpt2_state_dict(model_type)
        transposed = ["attn.c_attn.weight", "attn.c_proj.weight", "mlp.c_fc.weight", "mlp.c_proj.weight"]
        keys_hf = [k for k in sd_hf if not k.endswith(".attn.masked_bias") and not k.endswith(".attn.bias")]
        keys = [k for k in sd if not k.endswith(".attn.bias")]
        assert len(keys_hf) == len(keys), f"mismatched keys: {len(keys_hf)} != {len(keys)}"
        with torch.no_grad():
            for k in keys_hf:
                if any(k.endswith(w) for w in transposed):
                    # HF uses Conv1D modules: [in, out] weights
                    assert sd_hf[k].shape[::-1] == sd[k].shape
                    sd[k].copy_(sd_hf[k].t())
                else:
                    assert sd_hf[k].shape == sd[k].shape
                    sd[k].copy_(sd_hf[k])
        return model

    def optimizer_groups(self, weight_decay):
        """nanoGPT grouping: every >=2D tensor decays, biases/LayerNorms do not."""
        param_dict = {pn: p for pn, p in self.named_parameters() if p.requires_grad}
        decay_params = [p for n, p in param_dict.items() if p.dim() >= 2]
        nodecay_params = [p for n, p in param_dict.items() if p.dim() < 2]
        return [
            {"params": decay_params, "weight_decay": weight_decay},
            {"params": nodecay_params, "weight_decay": 0.0},
        ]

    def configure_optimizers(self, weight_decay, learning_rate, betas, device_type, store=None):
        """Two AdamW groups; on MI355X the optimizer is our fused flat HIP AdamW.

        With ``store`` (a ``FlatParamStore``) the fused flat optimizer is
        returned; without it a torch AdamW (``fused=True`` on GPU when available)
        is built, exactly like nanoGPT.
        """
        optim_groups = self.optimizer_groups(weight_decay)
        num_decay_params = sum(p.numel() for p in optim_groups[0]["params"])
        num_nodecay_params = sum(p.numel() for p in optim_groups[1]["params"])
        print(f"num decayed parameter tensors: {len(optim_groups[0]['params'])}, "
              f"with {num_decay_params:,} parameters")
        print(f"num non-decayed parameter tensors: {len(optim_groups[1]['params'])}, "
              f"with {num_nodecay_params:,} parameters")
        if store is not None:
            from ..optim.fused_adamw import FusedAdamW
            optimizer = FusedAdamW(store, optim_groups, lr=learning_rate, betas=betas)
            print(f"using fused AdamW: True (flat HIP kernel, {store.numel:,} elements)")
            return optimizer
        fused_available = "fused" in inspect.signature(torch.optim.AdamW).parameters
        use_fused = fused_available and device_type == "cuda"
        extra_args = dict(fused=True) if use_fused else dict()
        optimizer = torch.optim.AdamW(optim_groups, lr=learning_rate, betas=betas, **extra_args)
        print(f"using fused AdamW: {use_fused}")
        return optimizer

    def flops_per_token(self, seq_len=None):
        """nanoGPT's PaLM-appendix estimate: 6N + 12·L·H·Q·T (fwd+bwd)."""
        N = self.get_num_params()
        cfg = self.config
        L, H, Q, T = cfg.n_layer, cfg.n_head, cfg.n_embd // cfg.n_head, seq_len or cfg.block_size
        return 6 * N + 12 * L * H * Q * T

    def estimate_mfu(self, fwdbwd_per_iter, dt, peak_flops=MI355X_BF16_PEAK_FLOPS):
        """Model flops utilization in units of MI355X bf16 dense peak (not A100's 312 TF)."""
        T = self.config.block_size
        flops_per_fwdbwd = self.flops_per_token() * T
        flops_per_iter = flops_per_fwdbwd * fwdbwd_per_iter
        flops_achieved = flops_per_iter * (1.0 / dt)  # per second
        return flops_achieved / peak_flops

    @torch.no_grad()
    def generate(self, idx, max_new_tokens, temperature=1.0, top_k=None):
        """Autoregressive sampling: crop context, last-token logits / temperature,
        optional top-k, softmax, multinomial, append."""
        for _ in range(max_new_tokens):
            # if the sequence context is growing too long we must crop it at block_size
            idx_cond = idx if idx.size(1) <= self.config.block_size else idx[:, -self.config.block_size:]
            logits, _ = self(idx_cond)
            logits = logits[:, -1, :] / temperature
            if top_k is not None:
                v, _ = torch.topk(logits, min(top_k, logits.size(-1)))
                logits[logits < v[:, [-1]]] = -float("Inf")
            probs = torch.softmax(logits, dim=-1)
            idx_next = torch.multinomial(probs, num_samples=1)
            idx = torch.cat((idx, idx_next), dim=1)
        return idx

    @torch.no_grad()
    def generate_cached(self, idx, max_new_tokens, temperature=1.0, top_k=None, use_graph=None, decoder=None):
        """``generate`` with per-layer KV caches: the prompt is encoded once and every
        new token runs one position through the model (a replayed HIP graph on the GPU;
        ``runtime/decode.py``).  Same sampling; falls back to ``generate`` when prompt +
        new tokens exceed block_size."""
        from ..runtime.decode import generate_cached
        return generate_cached(self, idx, max_new_tokens, temperature=temperature, top_k=top_k, use_graph=use_graph,
                               decoder=decoder)
