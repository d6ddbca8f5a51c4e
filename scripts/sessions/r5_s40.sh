# weight-grad epilogue: fp32 atomics vs stored partials + ordered reduce, GPT-2 shapes
scripts/gpu_session.sh \
 "wg_det|300|python -u scripts/debug/wgrad_det_ab.py"
