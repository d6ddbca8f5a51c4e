# v5 hand-over fix + workgroup order A/B + K/V traffic probe
scripts/gpu_session.sh \
 "t_flash|400|python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'flash'" \
 "ab_order|300|python -u scripts/attn_ab.py --fwd 'v4:fwd=v4;v5:fwd=v5,order=0;v5o2:fwd=v5,order=2;v5o1:fwd=v5,order=1' --bwd 'v3:bwd=v3,order=0;v3o2:bwd=v3,order=2;v3o1:bwd=v3,order=1' --rounds 7" \
 "ab_kvshared|240|NSA_KERNEL_LIB=build/variants/kvshared/libnsa_kernels.so python -u scripts/attn_ab.py --fwd 'v5:fwd=v5,order=0;v5o2:fwd=v5,order=2' --bwd 'v3:bwd=v3' --rounds 5"
