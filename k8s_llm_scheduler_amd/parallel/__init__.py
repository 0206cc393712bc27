from .comm import TPGroup, init_from_env  # noqa: F401
