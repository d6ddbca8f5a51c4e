scripts/gpu_session.sh \
 "r6_v7_tests|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'flash and v7'" \
 "r6_ab_v7|200|python -u scripts/attn_ab.py --fwd 'v5:fwd=v5;v7:fwd=v7' --bwd v3:bwd=v3 --rounds 9 --iters 5"
