"""FedNAS local search trainer (reference: `mpi_p2p_mp/fednas/FedNASTrainer.py`): on each
client, alternate a DARTS architecture step (Adam on the alphas from the validation split —
first order, or the unrolled second-order gradient with ``unrolled: true``, Architect in
``models/cv/darts_architect.py``) with an SGD weight step (train split); in ``stage == "train"``
only weights move.
The model is ``models.cv.darts.Network``; alphas live in the state dict so the FedAvg
aggregator averages weights and architecture together."""
import logging

import torch
import torch.nn as nn

from ..core.alg_frame.client_trainer import ClientTrainer


class ModelTrainerNAS(ClientTrainer):
    def get_model_params(self):
        return {k: v.detach().cpu().clone() for k, v in self.model.state_dict().items()}

    def set_model_params(self, model_parameters):
        self.model.load_state_dict(model_parameters)

    def train(self, train_data, device, args=None):
        args = args or self.args
        model = self.model.to(device)
        model.train()
        crit = nn.CrossEntropyLoss()
        w_opt = torch.optim.SGD(model.weight_parameters(), lr=float(args.learning_rate),
                                momentum=float(getattr(args, "momentum", 0.9) or 0.9),
                                weight_decay=float(getattr(args, "weight_decay", 3e-4) or 3e-4))
        from ..models.cv.darts_architect import Architect
        if getattr(self, "_architect", None) is None or self._architect.model is not model:
            self._architect = Architect(model, args)   # keeps its Adam state across rounds, like the reference
        unrolled = bool(getattr(args, "unrolled", False))
        eta = float(args.learning_rate)
        search = str(getattr(args, "stage", "search")) == "search"
        batches = list(train_data)
        # reference splits each local shard into train / validation halves for the bilevel step
        half = max(1, len(batches) // 2) if search and len(batches) > 1 else len(batches)
        trn, val = batches[:half], batches[half:] or batches[:half]
        losses = []
        for _ in range(int(args.epochs)):
            for i, (x, y) in enumerate(trn):
                x, y = x.to(device), y.to(device)
                if search:   # first-order or unrolled second-order α step (models/cv/darts_architect.py)
                    vx, vy = val[i % len(val)]
                    self._architect.step(x, y, vx.to(device), vy.to(device), eta, w_opt, unrolled=unrolled)
                w_opt.zero_grad(set_to_none=True)
                loss = crit(model(x), y)
                loss.backward()
                nn.utils.clip_grad_norm_(model.weight_parameters(), float(getattr(args, "grad_clip", 5.0)))
                w_opt.step()
                losses.append(loss.detach())
        if losses:
            self.last_loss = float(torch.stack(losses).mean())
        logging.debug("client %s genotype %s", self.id, model.genotype())
        return getattr(self, "last_loss", None)

    @torch.no_grad()
    def test(self, test_data, device, args=None):
        model = self.model.to(device)
        model.eval()
        correct = total = 0
        loss = 0.0
        for x, y in test_data:
            x, y = x.to(device), y.to(device)
            out = model(x)
            loss += float(nn.functional.cross_entropy(out, y, reduction="sum"))
            correct += int((out.argmax(1) == y).sum())
            total += y.numel()
        return {"test_correct": correct, "test_total": total, "test_loss": loss}
