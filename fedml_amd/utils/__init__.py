from .logging import LoggerCreator
from .context import raise_error_and_retry, get_lock

__all__ = ["LoggerCreator", "raise_error_and_retry", "get_lock"]
