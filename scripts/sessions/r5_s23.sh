# chunked sorted embedding backward: tests, A/B at three shapes, headline bench
scripts/gpu_session.sh \
 "t_emb|300|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k 'embedding or deterministic'" \
 "ab_gpt2_b120|120|python -u scripts/emb_bwd_ab.py --B 120 --T 1024" \
 "ab_gpt2_b16|120|python -u scripts/emb_bwd_ab.py --B 16 --T 1024" \
 "ab_char|120|python -u scripts/emb_bwd_ab.py --B 64 --T 256 --V 56 --C 384" \
 "bench|400|python -u bench.py --steps 10 --warmup 3"
