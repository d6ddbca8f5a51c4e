# round 6: overlapped epilogue as a runtime policy (auto from K = 3072) and the GELU lookups
# batched per fragment row: GEMM tests, A/Bs on the training shapes, char shapes, bench
scripts/gpu_session.sh \
 "r6_t_gemm|300|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py" \
 "r6_ovl_ab2|400|python -u scripts/gemm_nt_ab.py --ovls 1,2 --shapes c_attn,attn.c_proj,mlp.c_proj,c_attn.dx,c_fc.dx --rounds 9" \
 "r6_grow_ab|300|python -u scripts/gemm_nt_ab.py --alt-lib build/variants/growoff/libnsa_kernels.so --epi --shapes c_fc --rounds 9" \
 "r6_bench20d|300|python -u bench.py --steps 20 --warmup 5" \
 "r6_char_gemm|300|python -u scripts/gemm_nt_ab.py --m 16384 --shapes 1152x384,384x384,1536x384,384x1536,384x1152 --rounds 7 --reps 20 --small"
