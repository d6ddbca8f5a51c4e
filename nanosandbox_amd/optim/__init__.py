from .flat import FlatParamStore  # noqa: F401
from .fused_adamw import FusedAdamW  # noqa: F401
