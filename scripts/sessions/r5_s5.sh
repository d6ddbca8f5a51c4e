# LayerNorm split-plane input probe; fixed CE ignored-row overflow; dK/dV pipelined pair A/B
scripts/gpu_session.sh \
 "probe_lnsplit|120|python -u scripts/debug/ln_split_probe.py" \
 "t_fix|300|python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_train_gpu.py -k 'many_rows or fixup or lm_head or dtype_contract'" \
 "ab_bwd5|300|python -u scripts/attn_ab.py --fwd 'v4:fwd=v4' --bwd 'v3:bwd=v3;v4:bwd=v4;v5:bwd=v5' --rounds 7"
