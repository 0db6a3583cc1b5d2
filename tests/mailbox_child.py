"""Child process of tests/test_device_mailbox_gpu.py: opens the server's mailbox from its IPC descriptor,
checks the published global model and writes its upload slot."""
import sys

import torch

from fedml_amd.core.distributed.communication.serialization import decode
from fedml_amd.cross_silo.device_mailbox import SiloMailbox


def main(path, slot):
    desc = decode(open(path, "rb").read())
    box = SiloMailbox(desc, slot)
    P = box.P
    mine = torch.empty(P, device="cuda")
    box.read_global(mine)
    want = torch.arange(P, dtype=torch.float32, device="cuda") * 0.5
    assert torch.equal(mine, want), float((mine - want).abs().max())
    box.write_upload(mine * (slot + 2), 10.0 * (slot + 1))
    print("child ok", slot, flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
