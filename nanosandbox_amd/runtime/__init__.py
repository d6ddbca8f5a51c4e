"""Host-side runtime pieces: HIP-graph capture of the training micro-step."""

from .hipgraph import MicroStepGraph, graph_capture_supported

__all__ = ["MicroStepGraph", "graph_capture_supported"]
