from .configurator import apply_overrides, config_keys, parse_argv  # noqa: F401
from .defaults import TRAIN_DEFAULTS  # noqa: F401
