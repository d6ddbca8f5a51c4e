scripts/gpu_session.sh "t_f16fix|200|python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_fp16_gpu.py -k 'fixup_rows'"
