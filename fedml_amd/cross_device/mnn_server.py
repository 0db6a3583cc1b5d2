"""``fedml_amd.cross_device.ServerMNN`` (reference: `cross_device/mnn_server.py:6-28`)."""
from .server_mnn import ServerMNN  # noqa: F401
