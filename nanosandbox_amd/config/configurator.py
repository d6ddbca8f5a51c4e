"""nanoGPT-compatible "poor man's configurator".

Behavioural contract (upstream nanoGPT ``configurator.py``
pulled in by reference ``notebooks/colab_nanoGPT_companion.ipynb:39,70-79``):

* an argv item without ``=`` is a config file: it must not start with ``--``;
  its text is printed and executed into the config namespace;
* ``--key=value`` overrides an *existing* key; the value goes through
  ``ast.literal_eval`` and falls back to the raw string; the parsed value must
  have exactly the type of the current value (so ``--dropout=0`` is rejected
  because ``0`` is an int and ``dropout`` a float);
* an unknown key raises ``ValueError("Unknown config key: <key>")``.

Unlike upstream this is a function over a dict, so it can be unit tested and
reused by ``train.py``, ``sample.py`` and ``bench.py`` without ``exec``-ing a
module file into ``globals()``.
"""

from __future__ import annotations

import sys
from ast import literal_eval
from typing import Iterable, MutableMapping


def _exec_config_file(path: str, namespace: MutableMapping, verbose: bool) -> None:
    with open(path) as f:
        src = f.read()
    if verbose:
        print(f"Overriding config with {path}:")
        print(src)
    # Config files are plain Python assigning module-level names; execute them
    # against a scratch namespace seeded with the current values, then copy
    # back every simple-typed name (matches nanoGPT, which exec's into globals).
    scratch = dict(namespace)
    exec(compile(src, path, "exec"), scratch)  # noqa: S102 - config files are code by contract
    for k, v in scratch.items():
        if k.startswith("_") or k == "__builtins__":
            continue
        if isinstance(v, (int, float, bool, str)) or k in namespace:
            namespace[k] = v


def apply_overrides(namespace: MutableMapping, argv: Iterable[str], verbose: bool = True) -> MutableMapping:
    """Apply nanoGPT configurator semantics for ``argv`` onto ``namespace``."""
    for arg in argv:
        if "=" not in arg:
            # assume it's the name of a config file
            assert not arg.startswith("--"), f"config file argument must not start with '--': {arg}"
            _exec_config_file(arg, namespace, verbose)
        else:
            # assume it's a --key=value argument
            assert arg.startswith("--"), f"override must look like --key=value: {arg}"
            key, val = arg.split("=", 1)
            key = key[2:]
            if key in namespace:
                try:
                    # attempt to eval it (e.g. if bool, number, etc)
                    attempt = literal_eval(val)
                except (SyntaxError, ValueError):
                    # if that goes wrong, just use the string
                    attempt = val
                # ensure the types match ok
                if type(attempt) != type(namespace[key]):  # noqa: E721 - exact type check is the contract
                    raise AssertionError(
                        f"type mismatch for --{key}: got {type(attempt).__name__} "
                        f"({attempt!r}), expected {type(namespace[key]).__name__}"
                    )
                if verbose:
                    print(f"Overriding: {key} = {attempt}")
                namespace[key] = attempt
            else:
                raise ValueError(f"Unknown config key: {key}")
    return namespace


def config_keys(namespace: MutableMapping) -> list:
    """The keys nanoGPT treats as configuration: public int/float/bool/str values."""
    return [k for k, v in namespace.items() if not k.startswith("_") and isinstance(v, (int, float, bool, str))]


def parse_argv(defaults: dict, argv=None, verbose: bool = True) -> dict:
    ns = dict(defaults)
    apply_overrides(ns, sys.argv[1:] if argv is None else argv, verbose=verbose)
    return ns
