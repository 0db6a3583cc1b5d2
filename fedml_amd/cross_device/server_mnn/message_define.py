from ...cross_silo.message_define import MyMessage  # same protocol ids (reference server_mnn/message_define.py)
