"""nanoGPT's configurator, for scripts that ``exec(open('configurator.py').read())``.

Applies ``sys.argv[1:]`` (config files and ``--key=value`` overrides) to the
caller's globals with nanoGPT's exact semantics; the implementation lives in
``nanosandbox_amd.config.configurator``.
"""
import sys as _sys

from nanosandbox_amd.config.configurator import apply_overrides as _apply_overrides

_apply_overrides(globals(), _sys.argv[1:])
