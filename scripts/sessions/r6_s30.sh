# round 6: GELU forward rows 4-7 deferred on the per-row lookup path (GDEF), as a variant
V=build/variants/gdef1/libnsa_kernels.so
scripts/gpu_session.sh \
 "r6_t_gdef|400|env NSA_KERNEL_LIB=$V python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_train_gpu.py" \
 "r6_gdef_ab|400|python -u scripts/gemm_nt_ab.py --alt-lib $V --epi --shapes c_fc --rounds 9"
