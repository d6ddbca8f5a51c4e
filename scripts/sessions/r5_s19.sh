# forward v5 variants (row sums as f32 adds; Q pre-scaled): back-to-back on one box, each
# against v4 inside its own process
scripts/gpu_session.sh \
 "ab_v5main|200|python -u scripts/attn_ab.py --fwd 'v4:fwd=v4;v5:fwd=v5' --bwd 'v3:bwd=v3' --rounds 11" \
 "ab_v5rs0|200|NSA_KERNEL_LIB=build/variants/fwd5rs0/libnsa_kernels.so python -u scripts/attn_ab.py --fwd 'v4:fwd=v4;v5:fwd=v5' --bwd 'v3:bwd=v3' --rounds 11" \
 "ab_v5qs1|200|NSA_KERNEL_LIB=build/variants/fwd5qs1/libnsa_kernels.so python -u scripts/attn_ab.py --fwd 'v4:fwd=v4;v5:fwd=v5' --bwd 'v3:bwd=v3' --rounds 11" \
 "ab_v5rs0qs1|200|NSA_KERNEL_LIB=build/variants/fwd5rs0qs1/libnsa_kernels.so python -u scripts/attn_ab.py --fwd 'v4:fwd=v4;v5:fwd=v5' --bwd 'v3:bwd=v3' --rounds 11" \
 "ab_v5main2|200|python -u scripts/attn_ab.py --fwd 'v4:fwd=v4;v5:fwd=v5' --bwd 'v3:bwd=v3' --rounds 11"
