# fp16 kernels: numerics, bf16 regression, bench in both dtypes; forward v6 A/B; dQ pipelined
# (bwd v4) A/B; split-plane LayerNorm gradient bench A/B;
# the skip-tile probe library must FAIL the exact-structure tests (expected rc 1)
scripts/gpu_session.sh \
 "t_new|300|python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'many_rows or raw_nan or exact_structure or split or pair_matches'" \
 "ab_bwd4|300|python -u scripts/attn_ab.py --fwd 'v4:fwd=v4' --bwd 'v3:bwd=v3;v4:bwd=v4' --rounds 7" \
 "ab_v6|300|python -u scripts/attn_ab.py --fwd 'v4:fwd=v4;v5:fwd=v5;v6:fwd=v6;v1:fwd=v1' --bwd 'v3:bwd=v3' --rounds 7" \
 "t_fp16|400|python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_fp16_gpu.py" \
 "probe_skiptile|200|NSA_KERNEL_LIB=build/variants/skiptile/libnsa_kernels.so python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'exact_structure and v4 and fwd'" \
 "t_bf16|600|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_optim_gpu.py" \
 "bench_bf16|300|python -u bench.py --steps 10 --warmup 3" \
 "bench_nosplit|300|NSA_LN_SPLIT=0 python -u bench.py --steps 10 --warmup 3" \
 "bench_bwd4|300|NSA_FLASH_BWD=v4 python -u bench.py --steps 10 --warmup 3" \
 "bench_fp16|300|python -u bench.py --steps 10 --warmup 3 --dtype float16"
