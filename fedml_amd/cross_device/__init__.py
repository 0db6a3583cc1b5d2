"""Cross-device FL (BeeHive): the server side; devices exchange model FILES (MNN or
safetensors) through the MQTT+blob-store transport."""
from .model_codec import MNNCodec, SafetensorsCodec, get_codec, load_indexed, model_to_indexed
from .server_mnn import ServerMNN
