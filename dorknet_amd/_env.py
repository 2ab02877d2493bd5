"""Environment switches read on the issue path.

The layers consult their DORKNET_* switches on every call (~250 lookups per training step);
``os.environ.get`` encodes the key and decodes the value each time (~1.2 us).  ``getenv``
reads the same mapping's backing dict with a pre-encoded key, so a switch changed at run
time (``os.environ[...] = ...``, pytest's monkeypatch) is still seen on the next call.
"""
from __future__ import annotations

import os

_DATA = getattr(os.environ, "_data", None)
_KEYS: dict = {}


def getenv(name: str, default=None):
    """os.environ.get(name, default), without the per-call key encoding."""
    if _DATA is None:
        return os.environ.get(name, default)
    k = _KEYS.get(name)
    if k is None:
        k = _KEYS[name] = os.fsencode(name)
    v = _DATA.get(k)
    return default if v is None else os.fsdecode(v)


def enabled(name: str) -> bool:
    """A default-on switch: off only when set to "0"."""
    return getenv(name, "1") != "0"
