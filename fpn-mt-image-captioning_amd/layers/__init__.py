from ._misc import *  # noqa: F401,F403  (mirrors the reference's layers/__init__.py)
