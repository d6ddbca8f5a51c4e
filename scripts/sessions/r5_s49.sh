scripts/gpu_session.sh \
 "t_ckpt|300|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'checkpointing or fused_resid'"
