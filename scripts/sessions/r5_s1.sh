scripts/gpu_session.sh \
 "t_optim|400|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_optim_gpu.py tests/test_train_gpu.py tests/test_gemm_gpu.py -k 'optim or dtype or fp16 or deterministic or bias'" \
 "t_flash|500|python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'flash'" \
 "ab_main|240|python -u scripts/attn_ab.py --fwd 'v4:fwd=v4;v5:fwd=v5' --bwd 'v3:bwd=v3' --rounds 7" \
 "ab_q1|240|NSA_KERNEL_LIB=build/variants/fwd5q1/libnsa_kernels.so python -u scripts/attn_ab.py --fwd 'v4:fwd=v4;v5:fwd=v5' --bwd 'v3:bwd=v3' --rounds 7" \
 "ab_rs0|240|NSA_KERNEL_LIB=build/variants/fwd5rs0/libnsa_kernels.so python -u scripts/attn_ab.py --fwd 'v4:fwd=v4;v5:fwd=v5' --bwd 'v3:bwd=v3' --rounds 7" \
 "bench|300|python -u bench.py --steps 10 --warmup 3"
