scripts/gpu_session.sh \
 "t_drop|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py tests/test_train_gpu.py -k 'dropout or layernorm or split or train'" \
 "t_all|1000|python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests/"
