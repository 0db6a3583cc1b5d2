"""Same-node device data plane for cross-silo model traffic (BASELINE config 5 on one MI355X node).

The reference moves every model between the server and the silo masters as a pickled / JSON state dict
over the network transport (``cross_silo/hierarchical/client_master_manager.py:239-249``): for ViT-B/16
that is 344 MB per message, serialised on the host, twice per silo and round. When the server and the
silo masters run on the same node, the payloads never need to leave HBM: the server exports two device
buffers through HIP IPC (``hipIpcGetMemHandle`` via torch's CUDA-IPC storage sharing; dmabuf mode,
``HSA_ENABLE_IPC_MODE_LEGACY=0``):

    glob  [P]           the current global model (flat fp32), written by the server after aggregation
    slot_s [P + 1]      one buffer per silo: its uploaded flat model ‖ its sample count

and the protocol messages (still on the TCP transport: handshake, round index, deadlines) carry only a
marker. A silo master copies ``glob`` into its client engine device-to-device (peer access over xGMI
when it sits on another GPU) and writes its silo average into its slot; the server aggregates the
slots with one FedAvg kernel over their stack. Every buffer is its own allocation and a silo imports only the
global buffer and its own slot: an import of one 2.75 GB allocation (8 ViT-B/16 slots in one tensor) never
returned on this ROCm (scripts/ipc_probe.py: 2 x 344 MB imports in 0.22 s; 8 x 344 MB as one buffer hung, alone
as well as concurrently). Ordering is by message: a writer
synchronises its stream before it sends the message that tells the reader to look.

Genuine WAN deployments keep the network transport (``silo_transport`` unset)."""
import fcntl
import logging
import os
import tempfile
import time

import torch

KEY = "__devmail__"


def _share(t: torch.Tensor) -> dict:
    """IPC descriptor of a CUDA tensor (wire-safe: ints, bytes and bools only — no pickle)."""
    st = t.untyped_storage()
    dev, handle, size, off, rc, rc_off, ev, ev_sync = st._share_cuda_()
    return {"device": int(dev), "handle": bytes(handle), "size": int(size), "off": int(off), "rc": bytes(rc),
            "rc_off": int(rc_off), "ev": bytes(ev) if ev is not None else b"", "ev_sync": bool(ev_sync),
            "shape": list(t.shape), "stride": list(t.stride()), "soff": int(t.storage_offset()),
            "dtype": str(t.dtype).replace("torch.", "")}


def _open(d: dict) -> torch.Tensor:
    torch.cuda._lazy_init()
    st = torch.UntypedStorage._new_shared_cuda(d["device"], d["handle"], d["size"], d["off"], d["rc"], d["rc_off"],
                                               d["ev"] or None, d["ev_sync"])
    typed = torch.storage.TypedStorage(wrap_storage=st, dtype=getattr(torch, d["dtype"]), _internal=True)
    return torch._utils._rebuild_tensor(typed, d["soff"], tuple(d["shape"]), tuple(d["stride"]))


class ServerMailbox:
    def __init__(self, P: int, n_slots: int, device):
        self.P = int(P)
        self.glob = torch.zeros(self.P, dtype=torch.float32, device=device)
        self.slots = [torch.zeros(self.P + 1, dtype=torch.float32, device=device) for _ in range(int(n_slots))]

    def descriptor(self) -> dict:
        return {"P": self.P, "glob": _share(self.glob), "slots": [_share(t) for t in self.slots]}

    def publish(self, flat: torch.Tensor):
        """The next round's global model, visible to the silos once this returns."""
        self.glob.copy_(flat.reshape(-1))
        torch.cuda.synchronize(self.glob.device)

    def upload(self, slot: int):
        """(flat model view, sample count) of a silo's upload."""
        row = self.slots[int(slot)]
        return row[:self.P], row[self.P:]


class SiloMailbox:
    def __init__(self, desc: dict, slot: int):
        self.P = int(desc["P"])
        # one importer at a time on the node: the silo masters all receive the descriptor at once, and
        # concurrent imports of the same dmabuf-backed IPC handles were seen to stall (8 silos; 2 were fine)
        t0 = time.time()
        with open(os.path.join(tempfile.gettempdir(), "fedml_amd_ipc_open.lock"), "a+") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            try:
                self.glob = _open(desc["glob"])
                self.slot_buf = _open(desc["slots"][int(slot)])
                torch.cuda.synchronize()
            finally:
                fcntl.flock(lk, fcntl.LOCK_UN)
        logging.info("device mailbox opened in %.2f s (slot %d)", time.time() - t0, int(slot))
        self.slot = int(slot)

    def read_global(self, out: torch.Tensor):
        out.reshape(-1).copy_(self.glob)

    def write_upload(self, flat: torch.Tensor, n_samples: float):
        row = self.slot_buf
        row[:self.P].copy_(flat.reshape(-1))
        row[self.P:].fill_(float(n_samples))
        torch.cuda.synchronize(flat.device)
        torch.cuda.synchronize(self.slot_buf.device)


def marker(kind: str, **kw) -> dict:
    return {KEY: kind, **kw}


def is_marker(params) -> bool:
    return isinstance(params, dict) and KEY in params
