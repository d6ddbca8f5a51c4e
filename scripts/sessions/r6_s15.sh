# round 6: fp16 cross-entropy guard + the many-rows fix-up test at 1100 rows (grid 1024)
scripts/gpu_session.sh \
 "r6_t_guard|400|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_fp16_gpu.py tests/test_kernels_gpu.py tests/test_train_gpu.py -k 'lm_head or xent or loss or guard or train'"
