from .core import close, create, evaluate, train  # noqa: F401
