# fp16 cross-entropy: fused fp16 vs autocast-form gradients against fp32
scripts/gpu_session.sh \
 "xent16|200|python -u scripts/debug/xent_f16_vs_autocast.py"
