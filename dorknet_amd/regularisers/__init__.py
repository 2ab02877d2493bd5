from . import l2  # noqa: F401
