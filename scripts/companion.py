"""The reference's Colab companion (notebooks/colab_nanoGPT_companion.ipynb, SURVEY.md
§2.1 P2-P6, nb:27-131), as one offline script over this stack.

    python scripts/companion.py [--workdir /tmp/companion] [--steps setup,data,cpu,ddp]

Cells, in notebook order:
  setup (P2)  check the GPU and the installed packages (no pip: the image is offline),
              build the HIP kernels in-tree
  data  (P3)  prepare shakespeare_char and place train.bin/val.bin/meta.pkl under
              <workdir>/data/datasets/shakespeare_char (the PVC layout)
  cpu   (P4)  the notebook's CPU smoke: exactly its flags (nb:70-79)
  ddp   (P5)  the 2-process torchrun demo.  The notebook puts rank 1 on cuda:1, which
              does not exist on a 1-GPU runtime (SURVEY.md §2.1 note on P5); here the
              demo picks a world that works: 2 GPUs -> RCCL on cuda:0/1; 1 GPU -> both
              ranks on cuda:0 with gloo collectives (NSA_REHEARSAL_ONE_GPU=1); no GPU ->
              gloo on CPU.
  notes (P6)  where logs, checkpoints and tfevents went
"""

from __future__ import annotations

import argparse
import importlib
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def sh(cmd, env=None):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=ROOT, env=env)


def gpu_count() -> int:
    # device_count() does not initialise HIP on this image (safe before launching children)
    import torch

    return torch.cuda.device_count() if hasattr(torch, "cuda") else 0


def step_setup(a):
    ngpu = gpu_count()
    print(f"GPUs visible: {ngpu}")
    for mod in ("torch", "numpy", "tiktoken", "safetensors", "yaml"):
        try:
            m = importlib.import_module(mod)
            print(f"  {mod:12s} {getattr(m, '__version__', 'ok')}")
        except ImportError:
            print(f"  {mod:12s} missing (optional)" if mod in ("tiktoken",) else f"  {mod:12s} MISSING")
    if ngpu:
        sh([sys.executable, "-m", "nanosandbox_amd.build"])


def step_data(a):
    out = os.path.join(a.workdir, "data", "datasets", "shakespeare_char")
    sh([sys.executable, "-m", "nanosandbox_amd.data.prepare", "char", "--out", out])
    print("dataset files:", sorted(os.listdir(out)))


def _base_flags(a):
    return ["config/train_shakespeare_char.py", f"--data_dir={os.path.join(a.workdir, 'data', 'datasets')}",
            "--eval_interval=50", "--log_interval=1", "--block_size=128", "--batch_size=16", "--n_layer=2",
            "--n_head=2", "--n_embd=64", "--dropout=0.0", "--compile=False", "--dataset=shakespeare_char"]


def step_cpu(a):
    runs = os.path.join(a.workdir, "runs")
    sh([sys.executable, "train.py", *_base_flags(a), f"--out_dir={os.path.join(runs, 'cpu')}",
        f"--max_iters={a.cpu_iters}", f"--lr_decay_iters={a.cpu_iters}", "--device=cpu",
        f"--tensorboard_dir={os.path.join(runs, 'tb', 'cpu')}"])


def step_ddp(a):
    runs = os.path.join(a.workdir, "runs")
    ngpu = gpu_count()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if ngpu >= 2:
        device, mode = "cuda", "RCCL on cuda:0/1"
    elif ngpu == 1:
        device, mode = "cuda", "both ranks on cuda:0 (gloo collectives)"
        env["NSA_REHEARSAL_ONE_GPU"] = "1"
    else:
        device, mode = "cpu", "gloo on CPU"
    print(f"2-process demo: {mode}")
    sh([sys.executable, "-m", "torch.distributed.run", "--standalone", "--nproc_per_node=2", "train.py",
        *_base_flags(a), f"--out_dir={os.path.join(runs, 'ddp')}", f"--max_iters={a.ddp_iters}",
        f"--lr_decay_iters={a.ddp_iters}", f"--device={device}", "--gradient_accumulation_steps=2",
        f"--tensorboard_dir={os.path.join(runs, 'tb', 'ddp')}"], env=env)


def step_notes(a):
    runs = os.path.join(a.workdir, "runs")
    print(f"logs/checkpoints under {runs}: {sorted(os.listdir(runs)) if os.path.isdir(runs) else []}")
    print(f"tensorboard --logdir {os.path.join(runs, 'tb')}   (events written by nanosandbox_amd.utils.tfevents)")
    print("torchrun --standalone == the single-Pod topology; the multi-Pod StatefulSet is exercised by "
          "tests/test_orchestration.py::test_multipod_emulation")


STEPS = {"setup": step_setup, "data": step_data, "cpu": step_cpu, "ddp": step_ddp, "notes": step_notes}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--workdir", default="/tmp/companion")
    ap.add_argument("--steps", default="setup,data,cpu,ddp,notes")
    ap.add_argument("--cpu-iters", type=int, default=50)
    ap.add_argument("--ddp-iters", type=int, default=100)
    ap.add_argument("--clean", action="store_true")
    a = ap.parse_args(argv)
    if a.clean and os.path.isdir(a.workdir):
        shutil.rmtree(a.workdir)
    os.makedirs(a.workdir, exist_ok=True)
    for s in a.steps.split(","):
        print(f"\n=== {s} ===", flush=True)
        STEPS[s](a)
    return 0


if __name__ == "__main__":
    sys.exit(main())
