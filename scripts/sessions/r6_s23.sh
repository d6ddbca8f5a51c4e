# round 6: OVL2 as the default for every plain bf16 GEMM with K >= 128; tests, A/B, bench
V=build/variants/ovl1/libnsa_kernels.so
scripts/gpu_session.sh \
 "r6_t_gemm4|300|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py" \
 "r6_ovl_ab3|500|python -u scripts/gemm_nt_ab.py --alt-lib $V --alt-ovl 1 --ovls 2 --shapes c_attn,attn.c_proj,c_attn.dx,mlp.c_proj,c_fc.dx --rounds 9" \
 "r6_bench20g|300|python -u bench.py --steps 20 --warmup 5"
