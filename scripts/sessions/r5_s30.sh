# GPT-2 1.5B N = 1600 GEMMs: nt4 full width vs nt4 over 1536 columns + a 64-column strip
scripts/gpu_session.sh \
 "nt_tail|300|python -u scripts/debug/nt_tail_probe.py"
