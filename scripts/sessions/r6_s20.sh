# round 6: attention kernels under other LLVM scheduler strategies (max-ilp, iterative-minreg)
A="python -u scripts/attn_ab.py --fwd auto: --bwd v3:bwd=v3 --rounds 7 --iters 5"
V1=build/variants/fa_maxilp/libnsa_kernels.so
V2=build/variants/fa_minreg/libnsa_kernels.so
scripts/gpu_session.sh \
 "r6_sched_t|300|NSA_KERNEL_LIB=$V1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'flash and not dropout_statistics'" \
 "r6_ab_def_1|120|$A" "r6_ab_maxilp_1|120|NSA_KERNEL_LIB=$V1 $A" "r6_ab_minreg_1|120|NSA_KERNEL_LIB=$V2 $A" \
 "r6_ab_def_2|120|$A" "r6_ab_maxilp_2|120|NSA_KERNEL_LIB=$V1 $A" "r6_ab_minreg_2|120|NSA_KERNEL_LIB=$V2 $A"
