"""Decentralized worker demo (reference: `mpi_p2p_mp/decentralized_framework/*`): workers on a
symmetric ring topology exchange their local result with out-neighbours and start the next
iteration once every in-neighbour's value arrived; each result is the topology-weighted mix."""
from ...core.distributed import FedMLCommManager, Message
from ...core.distributed.topology import SymmetricTopologyManager

MSG_NEIGHBOR_RESULT = 1


class DecentralizedWorkerManager(FedMLCommManager):
    def __init__(self, args, comm, rank, size, backend, topology):
        super().__init__(args, comm, rank, size, backend)
        self.topology = topology
        self.iteration = 0
        self.value = float(rank)
        self.inbox_vals = {}
        self.history = []
        self.in_neighbors = topology.get_in_neighbor_idx_list(rank)
        self.out_neighbors = topology.get_out_neighbor_idx_list(rank)

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MSG_NEIGHBOR_RESULT, self.handle)

    def start(self):
        self.broadcast()

    def broadcast(self):
        for nb in self.out_neighbors:
            m = Message(MSG_NEIGHBOR_RESULT, self.rank, nb)
            m.add_params("value", self.value)
            m.add_params("iteration", self.iteration)
            self.send_message(m)

    def handle(self, msg):
        it = int(msg.get("iteration"))
        self.inbox_vals.setdefault(it, {})[msg.get_sender_id()] = float(msg.get("value"))
        cur = self.inbox_vals.get(self.iteration, {})
        if len(cur) < len(self.in_neighbors):
            return
        w = self.topology.get_in_neighbor_weights(self.rank)
        new = float(w[self.rank]) * self.value + sum(float(w[j]) * v for j, v in cur.items())
        self.inbox_vals.pop(self.iteration)
        self.value = new
        self.history.append(new)
        self.iteration += 1
        if self.iteration >= int(self.args.comm_round):
            self.finish()
            return
        self.broadcast()


def FedML_Decentralized_Demo_distributed(args, process_id, worker_number, comm, device=None, dataset=None,
                                         model=None, model_trainer=None, **_):
    topo = SymmetricTopologyManager(worker_number, 2)
    topo.generate_topology()
    backend = "LOOPBACK" if comm is not None else str(getattr(args, "backend", "TCP"))
    w = DecentralizedWorkerManager(args, comm, process_id, worker_number, backend, topo)
    w.start()
    w.run()
    return {"history": w.history, "value": w.value}
