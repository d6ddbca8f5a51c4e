"""nanosandbox_amd — an MI355X-native (gfx950 / CDNA4) nanoGPT DDP training stack.

Capabilities follow fxcawley/nanoSandbox (reference README.md:1-127): nanoGPT
training driven by ``train.py config/x.py --key=value``, single-Pod and
multi-Pod DDP topologies, checkpoint/resume, and a Kubernetes deployment.

The compute path is designed for MI355X rather than translated:

* hot ops are hand-written HIP kernels for gfx950 (``csrc/kernels``), loaded
  from an in-tree shared library (``nanosandbox_amd/lib``),
* parameters, gradients and optimizer state live in single flat HBM buffers so
  that the optimizer is one fused pass and gradient buckets are zero-copy views,
* data parallelism uses our own bucketed reducer over RCCL (torch ``nccl``
  backend) sized for the 7 point-to-point xGMI links of an MI355X node.
"""

__version__ = "0.1.0"

from .models.gpt import GPT, GPTConfig  # noqa: F401
