"""HS-FedAvg: exact-Shapley client valuation + top-φ selection + Fourier amplitude sharing
(fork feature; reference: `single_process/hs_fedavg/fedavg_api.py:19-478`, `hs_fft.py`).

Per round each client normalises every training batch's low-frequency amplitude spectrum
toward a running amplitude (seeded from the server's averaged ``amp_summary``; on device via
``ops.spectral``), returns its running amplitude with its weights; the server averages the
amplitudes, values the clients with the exhaustive-coalition estimator (accumulating:
``sv_i += …``), updates ``φ_i ← α·φ_i + β·sv_i`` and selects the next round's clients as the
top-K by φ (uniform ``np.random.seed(round)`` sampling while all φ are equal).
"""
import logging
import time

import torch

from ....ops.spectral import amplitude_normalize
from ..valuation_base import ValuedFedAvgBase, hs_fedavg_sampling


class HS_FedAvgAPI(ValuedFedAvgBase):
    def _client_sampling(self, round_idx, client_num_in_total, client_num_per_round, phi=None):
        return hs_fedavg_sampling(round_idx, client_num_in_total, client_num_per_round, phi)

    def _client_train(self, client, w, amp_summary=None):
        state = {"amp": amp_summary.clone() if amp_summary is not None else None}
        momentum = float(getattr(self.args, "amp_momentum", 0.1))
        L = float(getattr(self.args, "amp_band", 0.0))

        def hook(x):
            if x.dim() != 4:
                return x
            out, state["amp"] = amplitude_normalize(x, state["amp"], momentum, False, L)
            return out

        self.model_trainer.input_hook = hook
        try:
            w_out = client.train(w)
        finally:
            self.model_trainer.input_hook = None
        self._amp_locals.append(state["amp"])
        return w_out

    def train(self):
        K = int(self.args.client_num_in_total)
        alpha, beta = self.alpha, self.beta
        phi = [1.0 / K] * K
        sv = [(1 - alpha) / (K * beta)] * K
        phi_dict, res_dict, sv_dict, client_dict, time_dict = {}, {}, {}, {}, {}
        amp_summary = None
        w_global = self.model_trainer.get_model_params()
        for round_idx in range(int(self.args.comm_round)):
            idxs = self._client_sampling(round_idx, K, int(self.args.client_num_per_round), phi)
            self._amp_locals = []
            w_locals = self._train_clients(idxs, w_global, amp_summary=amp_summary)
            amps = [a for a in self._amp_locals if a is not None]
            if amps:
                amp_summary = torch.stack([a.to(amps[0].device) for a in amps]).mean(0)
            t0 = time.time()
            valuer = self._valuer(w_locals)
            round_sv = valuer.exact_reference_sv()
            client_dict[round_idx] = {}
            for i, cid in enumerate(idxs):
                m = valuer.metrics[1 << i]
                client_dict[round_idx][int(cid)] = m["correct"] / max(1.0, m["total"])
                sv[cid] += round_sv[i]
                phi[cid] = alpha * phi[cid] + beta * sv[cid]
            time_dict[round_idx] = time.time() - t0
            w_global = self._finish_round(round_idx, w_locals, res_dict)
            phi_dict[round_idx], sv_dict[round_idx] = list(phi), list(sv)
        self.amp_summary = amp_summary
        self._dump(phi=phi_dict, res=res_dict, sv=sv_dict, client=client_dict, time=time_dict)
        return w_global
