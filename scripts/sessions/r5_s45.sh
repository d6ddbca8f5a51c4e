# dgrad / wgrad of one layer: one stream vs the weight grad on a second stream
scripts/gpu_session.sh \
 "overlap|200|python -u scripts/debug/overlap_probe.py"
