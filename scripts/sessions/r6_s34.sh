# round 6: XDX / fp16 GELU' epilogues re-derive the lane id (no spill reloads); tests and XDX A/B
V=build/variants/xlane0/libnsa_kernels.so
scripts/gpu_session.sh \
 "r6_t_xlane|500|python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_fp16_gpu.py tests/test_kernels_gpu.py" \
 "r6_xlane_ab|400|python -u scripts/gemm_nt_ab.py --alt-lib $V --xdx --shapes lm_head.dx --rounds 7"
