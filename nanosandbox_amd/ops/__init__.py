"""Fused GPT ops: HIP kernels on gfx950, fp32 torch reference on CPU."""

from .functional import (  # noqa: F401
    rng_advance,
    rng_set,
    set_deterministic,
    add_layer_norm,
    attention,
    compute_weight,
    decode_attention,
    decode_linear,
    dropout,
    embedding,
    gelu,
    kv_append,
    layer_norm,
    layer_norm_pass,
    linear,
    lm_head_logits,
    lm_head_loss,
    mlp,
    sample_topk_,
)
