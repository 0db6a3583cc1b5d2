"""FedGAN local trainer (reference: `mpi_p2p_mp/fedgan/MyModelTrainer.py`): alternating
discriminator / generator Adam steps with BCE on real-vs-fake; the model is the
``MNISTGAN`` container so one state dict carries both nets and FedAvg averages each."""
import torch
import torch.nn as nn

from ..core.alg_frame.client_trainer import ClientTrainer


class ModelTrainerGAN(ClientTrainer):
    def get_model_params(self):
        return {k: v.detach().cpu().clone() for k, v in self.model.state_dict().items()}

    def set_model_params(self, model_parameters):
        self.model.load_state_dict(model_parameters)

    def train(self, train_data, device, args=None):
        args = args or self.args
        g, d = self.model.netg.to(device), self.model.netd.to(device)
        g.train()
        d.train()
        lr = float(getattr(args, "learning_rate", 2e-4))
        opt_g = torch.optim.Adam(g.parameters(), lr=lr, betas=(0.5, 0.999))
        opt_d = torch.optim.Adam(d.parameters(), lr=lr, betas=(0.5, 0.999))
        bce = nn.BCELoss()
        nz = g.nz
        hist = []
        for _ in range(int(args.epochs)):
            for x, _y in train_data:
                x = x.to(device).reshape(x.shape[0], 1, 28, 28)
                if x.min() >= 0:  # images in [0,1] → generator range [-1,1]
                    x = x * 2 - 1
                b = x.shape[0]
                ones = torch.ones(b, 1, device=device)
                zeros = torch.zeros(b, 1, device=device)
                z = torch.randn(b, nz, device=device)
                fake = g(z)
                opt_d.zero_grad(set_to_none=True)
                loss_d = bce(d(x), ones) + bce(d(fake.detach()), zeros)
                loss_d.backward()
                opt_d.step()
                opt_g.zero_grad(set_to_none=True)
                loss_g = bce(d(fake), ones)
                loss_g.backward()
                opt_g.step()
                hist.append(torch.stack([loss_d.detach(), loss_g.detach()]))
        if hist:
            m = torch.stack(hist).mean(0).tolist()
            self.last_loss = {"loss_d": m[0], "loss_g": m[1]}
        return getattr(self, "last_loss", None)

    @torch.no_grad()
    def test(self, test_data, device, args=None):
        """Discriminator accuracy on real vs generated samples (GAN has no label accuracy)."""
        g, d = self.model.netg.to(device), self.model.netd.to(device)
        g.eval()
        d.eval()
        correct = total = 0
        for x, _y in test_data:
            x = x.to(device).reshape(x.shape[0], 1, 28, 28)
            if x.min() >= 0:
                x = x * 2 - 1
            real = d(x) > 0.5
            fake = d(g(torch.randn(x.shape[0], g.nz, device=device))) <= 0.5
            correct += int(real.sum()) + int(fake.sum())
            total += 2 * x.shape[0]
        return {"test_correct": correct, "test_total": total, "test_loss": 0.0}
