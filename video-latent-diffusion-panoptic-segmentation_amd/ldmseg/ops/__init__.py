from . import native  # noqa: F401
from .native import load_library  # noqa: F401
