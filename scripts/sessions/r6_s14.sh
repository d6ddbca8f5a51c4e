# round 6: the fp16 cross-entropy fix-up cliff, fix-up grid 1024 (new) vs 64 (round 5)
scripts/gpu_session.sh \
 "r6_cliff_1024|300|python -u scripts/debug/xent_f16_cliff.py --fracs 0,0.001,0.01,0.05" \
 "r6_cliff_64|300|NSA_KERNEL_LIB=build/variants/fix64/libnsa_kernels.so python -u scripts/debug/xent_f16_cliff.py --fracs 0,0.001,0.01" \
 "r6_cliff_bf16|300|python -u scripts/debug/xent_f16_cliff.py --dtype bfloat16 --fracs 0,0.01" \
 "r6_t_xent16|300|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_fp16_gpu.py tests/test_kernels_gpu.py -k 'lm_head or xent or loss'"
