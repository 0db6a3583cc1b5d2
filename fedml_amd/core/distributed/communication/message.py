"""Message envelope (reference: `core/distributed/communication/message.py:5-80`).

Same public API and key names (``msg_type``, ``sender``, ``receiver``, ``model_params``, ...).
Serialisation is NOT pickle: ``to_bytes()`` writes a JSON header plus raw tensor blobs
(``serialization.py``), so model payloads travel as flat buffers.
"""
import json


class Message:
    MSG_ARG_KEY_OPERATION = "operation"
    MSG_ARG_KEY_TYPE = "msg_type"
    MSG_ARG_KEY_SENDER = "sender"
    MSG_ARG_KEY_RECEIVER = "receiver"

    MSG_OPERATION_SEND = "send"
    MSG_OPERATION_RECEIVE = "receive"
    MSG_OPERATION_BROADCAST = "broadcast"
    MSG_OPERATION_REDUCE = "reduce"

    MSG_ARG_KEY_MODEL_PARAMS = "model_params"
    MSG_ARG_KEY_MODEL_PARAMS_URL = "model_params_url"
    MSG_ARG_KEY_NUM_SAMPLES = "num_samples"
    MSG_ARG_KEY_CLIENT_INDEX = "client_idx"
    MSG_ARG_KEY_CLIENT_STATUS = "client_status"
    MSG_ARG_KEY_CLIENT_OS = "client_os"

    def __init__(self, type=0, sender_id=0, receiver_id=0):
        self.type = str(type)
        self.sender_id = sender_id
        self.receiver_id = receiver_id
        self.msg_params = {
            Message.MSG_ARG_KEY_TYPE: type,
            Message.MSG_ARG_KEY_SENDER: sender_id,
            Message.MSG_ARG_KEY_RECEIVER: receiver_id,
        }

    def init(self, msg_params):
        self.msg_params = msg_params
        self.type = str(msg_params.get(Message.MSG_ARG_KEY_TYPE, 0))
        self.sender_id = msg_params.get(Message.MSG_ARG_KEY_SENDER, 0)
        self.receiver_id = msg_params.get(Message.MSG_ARG_KEY_RECEIVER, 0)

    def init_from_json_string(self, json_string):
        self.init(json.loads(json_string))

    def init_from_json_object(self, json_object):
        self.init(dict(json_object))

    def get_sender_id(self):
        return self.sender_id

    def get_receiver_id(self):
        return self.receiver_id

    def add_params(self, key, value):
        self.msg_params[key] = value

    add = add_params

    def get_params(self):
        return self.msg_params

    def get(self, key, default=None):
        return self.msg_params.get(key, default)

    def get_type(self):
        return self.msg_params[Message.MSG_ARG_KEY_TYPE]

    def to_string(self):
        return self.msg_params

    def to_json(self):
        """JSON-only form (tensors must already be lists — the MQTT path of the reference)."""
        return json.dumps(self.msg_params)

    def to_bytes(self) -> bytes:
        from .serialization import encode_message
        return encode_message(self)

    @staticmethod
    def from_bytes(buf: bytes) -> "Message":
        from .serialization import decode_message
        return decode_message(buf)

    def get_content(self):
        return "{}".format(self.msg_params)

    def __repr__(self):
        keys = {k: (type(v).__name__ if not isinstance(v, (int, float, str, bool)) else v)
                for k, v in self.msg_params.items()}
        return f"Message({keys})"
