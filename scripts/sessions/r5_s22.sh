# probe the char_skew failure of the chunked embedding backward
scripts/gpu_session.sh \
 "probe|120|python -u scripts/debug/emb_chunk_probe.py"
