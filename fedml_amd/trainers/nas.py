"""FedNAS local trainer (reference: `mpi_p2p_mp/fednas/FedNASTrainer.py`).

``stage: search`` (``search()``, :43-165): on each client, alternate a DARTS architecture step (Adam on the
alphas from the validation split — first order, or the unrolled second-order gradient with
``unrolled: true``, Architect in ``models/cv/darts_architect.py``) with an SGD weight step (train split).
The model is ``models.cv.darts.Network`` (or the GDAS ``Network_GumbelSoftmax``); alphas live in the state
dict so the FedAvg aggregator averages weights and architecture together.

``stage: train`` (``train()``, :167-246): the genotype-built ``NetworkCIFAR`` trains its weights only — SGD
with cosine annealing over the local epochs (to ``learning_rate_min``), the auxiliary head's loss added
with ``auxiliary_weight``, drop-path probability ramped over the epochs, gradient clipping."""
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
        if str(getattr(args, "stage", "search")) == "train" and not hasattr(model, "arch_parameters"):
            return self._train_eval_net(model, train_data, device, args)
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

    def _train_eval_net(self, model, train_data, device, args):
        """``stage: train`` on the genotype network (FedNASTrainer.train / local_train)."""
        crit = nn.CrossEntropyLoss()
        epochs = int(args.epochs)
        opt = torch.optim.SGD(model.parameters(), lr=float(args.learning_rate),
                              momentum=float(getattr(args, "momentum", 0.9) or 0.9),
                              weight_decay=float(getattr(args, "weight_decay", 3e-4) or 3e-4))
        sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, float(epochs),
                                                           eta_min=float(getattr(args, "learning_rate_min", 0.001)))
        aux_w = float(getattr(args, "auxiliary_weight", 0.4))
        dpp = float(getattr(args, "drop_path_prob", 0.2))
        losses = []
        for ep in range(epochs):
            model.drop_path_prob = dpp * ep / max(1, epochs)
            for x, y in train_data:
                x, y = x.to(device), y.to(device)
                opt.zero_grad(set_to_none=True)
                logits, aux = model(x)
                loss = crit(logits, y)
                if aux is not None:
                    loss = loss + aux_w * crit(aux, y)
                loss.backward()
                nn.utils.clip_grad_norm_(model.parameters(), float(getattr(args, "grad_clip", 5.0)))
                opt.step()
                losses.append(loss.detach())
            sched.step()
        if losses:
            self.last_loss = float(torch.stack(losses).mean())
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
            if isinstance(out, tuple):   # NetworkCIFAR: (logits, auxiliary logits)
                out = out[0]
            loss += float(nn.functional.cross_entropy(out, y, reduction="sum"))
            correct += int((out.argmax(1) == y).sum())
            total += y.numel()
        return {"test_correct": correct, "test_total": total, "test_loss": loss}
