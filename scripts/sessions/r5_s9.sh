scripts/gpu_session.sh "probe_xent16|120|python -u scripts/debug/xent_f16_probe.py"
