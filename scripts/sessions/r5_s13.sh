# PMC: attention (round-5 defaults) and the LayerNorm bytes
scripts/gpu_session.sh \
 "pmc_attn|300|PMC_ATTN_ARGS='--rounds 1 --iters 2 --fwd auto:;v4:fwd=v4 --bwd v3:bwd=v3' bash scripts/pmc_attn.sh" \
 "pmc_ln|400|bash scripts/pmc_ln.sh"
