# round 6: forward variants trimmed to v1 / v5 (skiptile probe moved into v5, must FAIL:
# expected rc 1), selective MLP recompute (bitwise vs resident), 1.5B modes, bench
scripts/gpu_session.sh \
 "r6_t_flash|400|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp16_gpu.py -k 'flash or attention'" \
 "r6_probe_skiptile|200|NSA_KERNEL_LIB=build/variants/skiptile/libnsa_kernels.so python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'exact_structure and v5 and fwd'" \
 "r6_t_recompute|300|python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_train_gpu.py -k recompute" \
 "r6_xl_res_b|600|python -u bench.py --model gpt2-xl --micro-batch 60 --steps 2 --warmup 1 --calib-seconds 1" \
 "r6_xl_rm60|600|python -u bench.py --model gpt2-xl --recompute-mlp --micro-batch 60 --steps 2 --warmup 1 --calib-seconds 0" \
 "r6_xl_rm120|600|python -u bench.py --model gpt2-xl --recompute-mlp --micro-batch 120 --steps 2 --warmup 1 --calib-seconds 0" \
 "r6_bench20c|300|python -u bench.py --steps 20 --warmup 5"
