# deterministic mode at the headline shape (fused cross-entropy now kept there), twice: same loss bit for bit
scripts/gpu_session.sh \
 "det1|400|python -u bench.py --steps 4 --warmup 2 --deterministic" \
 "det2|400|python -u bench.py --steps 4 --warmup 2 --deterministic"
