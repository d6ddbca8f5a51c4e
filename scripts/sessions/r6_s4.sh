A="python -u scripts/attn_ab.py --fwd auto: --bwd v3:bwd=v3 --rounds 7 --iters 5"
V=build/variants/fa_slp/libnsa_kernels.so
scripts/gpu_session.sh \
 "r6_attn_tests|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'flash'" \
 "r6_ab_noslp_1|120|$A" "r6_ab_slp_1|120|NSA_KERNEL_LIB=$V $A" \
 "r6_ab_noslp_2|120|$A" "r6_ab_slp_2|120|NSA_KERNEL_LIB=$V $A" \
 "r6_ab_noslp_3|120|$A" "r6_ab_slp_3|120|NSA_KERNEL_LIB=$V $A"
