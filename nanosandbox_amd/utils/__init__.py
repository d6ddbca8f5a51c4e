from .checkpoint import load_checkpoint, load_model_state, save_checkpoint, strip_compile_prefix  # noqa: F401
from .lr import get_lr  # noqa: F401
from .metrics import MetricsLogger  # noqa: F401
