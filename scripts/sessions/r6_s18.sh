# round 6: the HBM copy roofline on this box (LayerNorm passes run 5.9-6.1 TB/s)
scripts/gpu_session.sh \
 "r6_hbm_copy|200|python -u scripts/debug/hbm_copy_probe.py" \
 "r6_membound|300|python -u scripts/membound_ab.py"
