scripts/gpu_session.sh "r6_xent_nan|200|python -u scripts/debug/xent_nan_map.py"
