# round 6: where the XENT GEMM's extra ~1 ms per call goes (probe build: no epilogue / no stores)
scripts/gpu_session.sh \
 "r6_xent_probe0|200|python -u scripts/gemm_nt_ab.py --alt-lib build/variants/probes/libnsa_kernels.so --xent --shapes lm_head --rounds 5 --reps 3" \
 "r6_xent_probe4|200|NSA_PROBE_XENT=4 python -u scripts/gemm_nt_ab.py --alt-lib build/variants/probes/libnsa_kernels.so --xent --shapes lm_head --rounds 5 --reps 3" \
 "r6_xent_probe5|200|NSA_PROBE_XENT=5 python -u scripts/gemm_nt_ab.py --alt-lib build/variants/probes/libnsa_kernels.so --xent --shapes lm_head --rounds 5 --reps 3"
