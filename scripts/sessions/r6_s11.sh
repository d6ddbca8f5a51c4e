# round 6: GELU' epilogue with the U loads issued ahead of each fragment row's stores
scripts/gpu_session.sh \
 "r6_t_gemm3|300|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py" \
 "r6_dgelu_ab|400|python -u scripts/gemm_nt_ab.py --alt-lib build/variants/growoff/libnsa_kernels.so --epi --shapes mlp.c_proj.dx,c_fc --rounds 9"
