"""Incremental decoding with per-layer KV caches, one token's forward replayed as a HIP graph.

nanoGPT's ``generate`` (reference ``sample.py`` -> ``model.generate``, SURVEY.md §2.3
U-M11/U-S1) runs the whole context through the model for every new token: O(T)
work per token for the projections and O(T^2) for attention, and at serving batch
sizes a few hundred tiny kernel launches per token whose host overhead dominates.

``Decoder`` keeps K and V of every layer in bf16 caches [B, H, block_size, D]
(``ops.kv_append``) and decodes one position at a time:

* ``prefill(idx)``: the prompt goes through the normal fused forward (flash
  attention over the prompt), each layer's K/V rows are written to the caches, and
  the last position's logits are returned;
* ``step(tok)``: embedding of the new token at position ``pos`` -> per layer
  residual-add+LN+c_attn -> append K/V + single-query attention over the cache
  (``ops.decode_attention``: split-K flash-decoding kernels) -> combine+c_proj ->
  residual-add+LN+c_fc+GELU -> c_proj -> ... -> residual-add+ln_f+lm_head (at batch
  1 each arrow's producer runs in the prologue of the next weight-streaming kernel).  ``pos`` lives in a device tensor
  that the step itself increments, so on the GPU the whole step is captured once
  as a ``torch.cuda.CUDAGraph`` and replayed per token (one launch per token).

Sampling (temperature, top-k, multinomial) is nanoGPT's distribution, drawn on the
device by one kernel (``ops.sample_topk_``: radix-select threshold, softmax mass, scan,
counter-hash uniform) that writes the id straight into the fed-token buffer and into
``gen`` at the device position.  ``run(n)`` captures step + sampling as one graph, so
n tokens are n replays with no host round trip.
The caches hold at most ``block_size`` positions; ``GPT.generate_cached`` falls
back to the recompute loop when prompt + new tokens exceed that (nanoGPT crops the
context there, which a cache cannot do without re-encoding).
"""

from __future__ import annotations

import torch

from .. import ops


class Decoder:
    def __init__(self, model, batch_size: int, max_len: int | None = None, use_graph: bool | None = None):
        self.model = model
        cfg = model.config
        self.B = batch_size
        self.T = max_len or cfg.block_size
        assert self.T <= cfg.block_size, "caches cannot exceed the position-embedding table"
        self.H = cfg.n_head
        self.D = cfg.n_embd // cfg.n_head
        p = model.lm_head.weight
        self.device = p.device
        self.dtype = model.compute_dtype
        self.rdtype = model.residual_dtype
        shape = (batch_size, self.H, self.T, self.D)
        self.kc = [torch.zeros(shape, device=self.device, dtype=self.dtype) for _ in range(cfg.n_layer)]
        self.vc = [torch.zeros(shape, device=self.device, dtype=self.dtype) for _ in range(cfg.n_layer)]
        self.pos = torch.zeros(1, device=self.device, dtype=torch.int64)  # position of the token being fed
        self.tok = torch.zeros(batch_size, 1, device=self.device, dtype=torch.int64)
        # generated tokens by position: gen[:, p] is the token fed at position p
        self.gen = torch.zeros(batch_size, self.T + 1, device=self.device, dtype=torch.int64)
        self.salt = int(torch.randint(0, 2 ** 62, (1,)).item())  # sampling stream (torch.manual_seed governs)
        # per-call part of the sampling stream, read by the kernel at run time (so a captured
        # sampling graph, reused across generate calls, draws independent samples each call)
        self.salt_dev = torch.zeros(1, device=self.device, dtype=torch.int64)
        self.use_graph = (self.device.type == "cuda") if use_graph is None else use_graph
        if self.use_graph and not self.graph_capable(model):
            # the fused decode kernels cover head_dim 64, bf16 and V <= 53248; the fallback
            # ops read the position back to the host (pos.item()) or refuse wider vocabs,
            # which a captured graph cannot do: run those configs eagerly
            self.use_graph = False
        self.graph = None      # step(): logits only
        self.sgraphs = {}      # run(): step + sampling + token feedback, per (temperature, top_k)
        self.logits = None
        self.replays = 0
        # compute-dtype weight shadows (``param.compute``, what every op reads): a trained
        # model carries the optimizer's; a freshly loaded one would otherwise convert each
        # fp32 weight on every use (124M: ~750 MB of conversion traffic per token, and
        # inside the captured graph too).  Created here, dropped by ``release()``.
        self._shadowed = []
        if self.dtype != torch.float32:
            for prm in model.parameters():
                c = getattr(prm, "compute", None)
                if c is None or c.dtype != self.dtype:
                    prm.compute = prm.detach().to(self.dtype)
                    self._shadowed.append(prm)

    @staticmethod
    def graph_capable(model) -> bool:
        cfg = model.config
        return (cfg.n_embd // cfg.n_head == 64 and model.compute_dtype == torch.bfloat16
                and cfg.vocab_size <= 53248)

    def release(self):
        """Drop the weight shadows this decoder created and its captured graph."""
        for prm in self._shadowed:
            try:
                del prm.compute
            except AttributeError:
                pass
        self._shadowed = []
        self.graph = None
        self.sgraphs = {}

    # ------------------------------------------------------------------ layers
    def _prefill_layers(self, x):
        tr = self.model.transformer
        blocks = tr.h
        ln = blocks[0].ln_1
        x, h = ops.layer_norm_pass(x, ln.weight, ln.bias, out_dtype=ln.out_dtype)
        for i, block in enumerate(blocks):
            nxt = blocks[i + 1].ln_1 if i + 1 < len(blocks) else tr.ln_f
            attn, mlp = block.attn, block.mlp
            qkv = ops.linear(h, attn.c_attn.weight, attn.c_attn.bias)
            ops.kv_append(qkv, self.kc[i], self.vc[i], None, 0)
            y = ops.attention(qkv, attn.n_head, 0.0, False)
            y = ops.linear(y, attn.c_proj.weight, attn.c_proj.bias)
            x, h2 = ops.add_layer_norm(x, y, block.ln_2.weight, block.ln_2.bias)
            y = mlp(h2)
            x, h = ops.add_layer_norm(x, y, nxt.weight, nxt.bias)
        return h  # ln_f(x)

    def _decode_layers(self):
        """The token ``tok`` at position ``pos`` through the embedding, every block and the
        head -> fp32 logits [B, 1, V].

        Each linear's producer rides in its prologue at batch 1: the embedding and ln_1 in
        c_attn's (``ops.decode_embed_linear_ln``), the residual add + LayerNorm in c_attn /
        c_fc / lm_head (``ops.decode_linear_ln``), the flash-decoding combine in c_proj's
        (``decode_attention(combine=False)`` -> ``ops.decode_linear``); the K / V append
        rides in the attention kernel and bias / GELU in the GEMV epilogues: 5 launches
        per layer."""
        tr = self.model.transformer
        branch = None  # the previous sublayer's output, not yet added to the residual x
        for i, block in enumerate(tr.h):
            attn, mlp = block.attn, block.mlp
            ln1, ln2 = block.ln_1, block.ln_2
            if i == 0:
                x, qkv = ops.decode_embed_linear_ln(self.tok, self.pos, tr.wte.weight, tr.wpe.weight, ln1.weight,
                                                    ln1.bias, attn.c_attn.weight, attn.c_attn.bias, dtype=self.dtype,
                                                    res_dtype=self.rdtype, out_dtype=ln1.out_dtype)
            else:
                x, qkv = ops.decode_linear_ln(x, branch, ln1.weight, ln1.bias, attn.c_attn.weight, attn.c_attn.bias,
                                              out_dtype=ln1.out_dtype)
            y = ops.decode_attention(qkv, self.kc[i], self.vc[i], self.pos, attn.n_head, append=True, combine=False)
            y = ops.decode_linear(y, attn.c_proj.weight, attn.c_proj.bias)
            x, u = ops.decode_linear_ln(x, y, ln2.weight, ln2.bias, mlp.c_fc.weight, mlp.c_fc.bias, gelu=True,
                                        out_dtype=ln2.out_dtype)
            branch = ops.decode_linear(u, mlp.c_proj.weight, mlp.c_proj.bias)
        lnf = tr.ln_f
        _, logits = ops.decode_linear_ln(x, branch, lnf.weight, lnf.bias, self.model.lm_head.weight, None,
                                         out_f32=True, out_dtype=lnf.out_dtype, pos_inc=self.pos)
        return logits  # pos has advanced (by the head kernel itself on the fused path)

    @torch.no_grad()
    def prefill(self, idx: torch.Tensor) -> torch.Tensor:
        """Encode the prompt [B, T0]; returns the last position's logits [B, V] (fp32)."""
        B, T0 = idx.shape
        assert B == self.B and 1 <= T0 <= self.T
        tr = self.model.transformer
        x = ops.embedding(idx, tr.wte.weight, tr.wpe.weight, 0.0, False, dtype=self.rdtype, cdtype=self.dtype)
        h = self._prefill_layers(x)
        self.pos.fill_(T0)
        return ops.lm_head_logits(h[:, [-1], :], self.model.lm_head.weight)[:, 0]

    def _step_impl(self):
        return self._decode_layers()[:, 0]  # also advances pos

    @torch.no_grad()
    def step(self, tok: torch.Tensor) -> torch.Tensor:
        """Feed one token per sequence ([B] or [B, 1]) at the current position; returns
        the logits [B, V] for the next position (a view of a static buffer on the GPU)."""
        self.tok.copy_(tok.view(self.B, 1))
        if not self.use_graph:
            return self._step_impl()
        if self.graph is None:
            self._capture()
        self.graph.replay()
        self.replays += 1
        return self.logits

    def _warmup(self, fn):
        # outside any graph (lazy library init, GEMM tuner decisions for M = B), at the
        # current position without advancing it or changing the fed token: the captured
        # step rewrites the same cache rows when it runs
        tok = self.tok.clone()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                fn()
                self.pos.sub_(1)
                self.tok.copy_(tok)
        torch.cuda.current_stream().wait_stream(side)

    def _capture(self):
        self._warmup(self._step_impl)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):  # recorded, not executed: pos is unchanged
            self.logits = self._step_impl()

    def sample_into(self, logits, temperature, top_k):
        """Draw the next token of every row from ``logits`` [B, V] into ``tok`` and
        ``gen[:, pos]`` (device kernel on the GPU: ``ops.sample_topk_``)."""
        ops.sample_topk_(logits, temperature, top_k, self.salt, self.pos, self.tok, self.gen, salt_dev=self.salt_dev)

    def reseed(self):
        """A fresh sampling stream for the next generate call (torch.manual_seed governs)."""
        self.salt_dev.fill_(int(torch.randint(0, 2 ** 62, (1,)).item()))

    def _step_sample_impl(self, temperature, top_k):
        self.sample_into(self._step_impl(), temperature, top_k)  # pos is now p + 1

    @torch.no_grad()
    def run(self, n: int, temperature: float = 1.0, top_k: int | None = None):
        """Decode n tokens starting from ``self.tok`` at ``self.pos``: each step feeds the
        token, samples the next one and feeds it back on the device (one graph replay per
        token on the GPU, no host round trip).  Results land in ``self.gen``."""
        if not self.use_graph:
            for _ in range(n):
                self._step_sample_impl(temperature, top_k)
            return
        key = (float(temperature), top_k)
        g = self.sgraphs.get(key)
        if g is None:
            self._warmup(lambda: self._step_sample_impl(temperature, top_k))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._step_sample_impl(temperature, top_k)
            self.sgraphs[key] = g
        for _ in range(n):
            g.replay()
        self.replays += n

    @property
    def position(self) -> int:
        return int(self.pos.item())


def sample_next(logits: torch.Tensor, temperature: float = 1.0, top_k: int | None = None,
                generator: torch.Generator | None = None) -> torch.Tensor:
    """nanoGPT's sampling: logits / temperature, optional top-k, softmax, multinomial -> [B, 1]."""
    logits = logits.float() / temperature
    if top_k is not None:
        v, _ = torch.topk(logits, min(top_k, logits.size(-1)))
        logits = logits.masked_fill(logits < v[:, -1:], -float("Inf"))  # basic slicing: capturable
    probs = torch.softmax(logits, dim=-1)
    return torch.multinomial(probs, num_samples=1, generator=generator)


@torch.no_grad()
def generate_cached(model, idx: torch.Tensor, max_new_tokens: int, temperature: float = 1.0,
                    top_k: int | None = None, use_graph: bool | None = None,
                    decoder: "Decoder | None" = None) -> torch.Tensor:
    """``model.generate`` with KV caches: same sampling, one token's forward per new token.

    ``decoder``: a Decoder to reuse across calls (same batch size): its weight shadows and
    captured graphs survive, so ``sample.py``'s num_samples loop captures once.  The caller
    releases it; without one, a temporary decoder is built and released here."""
    B, T0 = idx.shape
    if max_new_tokens <= 0:
        return idx
    if T0 + max_new_tokens - 1 > model.config.block_size:
        # the caches hold block_size positions; nanoGPT crops the context beyond that
        return model.generate(idx, max_new_tokens, temperature=temperature, top_k=top_k)
    own = decoder is None or decoder.B != B
    dec = Decoder(model, B, max_len=model.config.block_size, use_graph=use_graph) if own else decoder
    try:
        dec.reseed()  # every call draws its own samples, also on a reused decoder / graph
        dec.sample_into(dec.prefill(idx), temperature, top_k)  # pos = T0: gen[:, T0]
        dec.run(max_new_tokens - 1, temperature, top_k)
        return torch.cat([idx, dec.gen[:, T0:T0 + max_new_tokens]], dim=1)
    finally:
        if own:
            dec.release()
