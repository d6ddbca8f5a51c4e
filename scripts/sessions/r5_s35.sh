# char-config GEMM shapes: weight-grad split sweep (wgrad4 vs ring64), NT kernels (nt4 vs small)
scripts/gpu_session.sh \
 "wg_small|300|python -u scripts/debug/wgrad_small_ab.py" \
 "nt_small|200|python -u scripts/debug/nt_small_ab.py"
