from .base import FuncProvider, Provider, Request, Response, StreamCallback  # noqa: F401
from .registry import Registry, UnknownModelError  # noqa: F401
