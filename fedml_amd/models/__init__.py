"""Model zoo (``fedml_amd.model`` alias)."""
from .model_hub import create

__all__ = ["create"]
