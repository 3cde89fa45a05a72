"""XML handlers (control layer).  Importing this package registers every element."""
from . import base, core, optimization  # noqa: F401
from .base import REGISTRY, make_handler  # noqa: F401
