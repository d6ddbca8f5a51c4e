# strip kernel v2 (barrier-free register ring): numerics + ring depth sweep
scripts/gpu_session.sh \
 "t_strip|300|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'strip'" \
 "probe_d4|120|python -u scripts/debug/nt_tail_probe.py" \
 "probe_d2|120|env NSA_KERNEL_LIB=build/variants/strip_d2/libnsa_kernels.so python -u scripts/debug/nt_tail_probe.py" \
 "probe_d6|120|env NSA_KERNEL_LIB=build/variants/strip_d6/libnsa_kernels.so python -u scripts/debug/nt_tail_probe.py" \
 "probe_d8|120|env NSA_KERNEL_LIB=build/variants/strip_d8/libnsa_kernels.so python -u scripts/debug/nt_tail_probe.py"
