"""Reference-compatible alias: ``fedml.model`` (the reference package name) → ``fedml_amd.models``."""
from ..models import *  # noqa: F401,F403
from ..models import create  # noqa: F401
