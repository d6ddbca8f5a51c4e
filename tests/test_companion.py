"""The Colab-companion equivalent (scripts/companion.py, reference P2-P6) runs offline on CPU."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_companion_data_and_cpu_smoke(tmp_path):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "companion.py"), "--workdir", str(tmp_path),
                          "--steps", "data,cpu,notes", "--cpu-iters", "5"],
                         capture_output=True, text=True, timeout=600, env={**os.environ, "CUDA_VISIBLE_DEVICES": ""})
    assert out.returncode == 0, out.stderr[-2000:]
    assert "iter 4:" in out.stdout
    ds = tmp_path / "data" / "datasets" / "shakespeare_char"
    assert {"train.bin", "val.bin", "meta.pkl"} <= set(os.listdir(ds))
    assert os.path.isdir(tmp_path / "runs" / "tb" / "cpu")
