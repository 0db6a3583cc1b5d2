"""S-FedAvg: Shapley-valued client selection (fork feature; reference:
`single_process/s_fedavg/fedavg_api.py:24-653`).

Per round: sample clients with ``p ∝ exp(φ)`` (``sampling_filter == "exp"``) else uniformly;
train them with class-balanced CE and grad-clip 1.0; value them — Monte-Carlo permutation
Shapley when ``sv_approaching`` (stop when the last 3 updates moved < 0.005 or after K²
permutations), else the reference's exhaustive-coalition estimator — with the coalition score
being validation accuracy or the target label's F1 / recall / precision; then
``φ_i ← α·φ_i + β·sv_i`` and FedAvg. Coalition models are aggregated by one MFMA product and
evaluated in client-batched forwards (``core.valuation``).
"""
import logging
import time

import numpy as np

from ..valuation_base import ValuedFedAvgBase, s_fedavg_sampling


class S_FedAvgAPI(ValuedFedAvgBase):
    def _client_sampling(self, round_idx, client_num_in_total, client_num_per_round, phi=None, sampling_filter=None):
        return s_fedavg_sampling(round_idx, client_num_in_total, client_num_per_round, phi, sampling_filter)

    def train(self):
        K = int(self.args.client_num_in_total)
        alpha, beta = self.alpha, self.beta
        phi = [1.0 / K] * K
        sv = [(1 - alpha) / (K * beta)] * K
        phi_dict, res_dict, sv_dict, client_dict, time_dict = {}, {}, {}, {}, {}
        w_global = self.model_trainer.get_model_params()
        rng = np.random.RandomState((self.seed * 7919 + 17) & 0xFFFFFFFF)
        for round_idx in range(int(self.args.comm_round)):
            idxs = self._client_sampling(round_idx, K, int(self.args.client_num_per_round), phi,
                                         self.sampling_filter)
            w_locals = self._train_clients(idxs, w_global)
            t0 = time.time()
            valuer = self._valuer(w_locals)
            round_sv = valuer.monte_carlo_sv(rng) if self.sv_approaching else valuer.exact_reference_sv()
            valuer.ensure([1 << i for i in range(len(w_locals))])
            client_dict[round_idx] = {}
            for i, cid in enumerate(idxs):
                m = valuer.metrics[1 << i]
                client_dict[round_idx][int(cid)] = m["correct"] / max(1.0, m["total"])
                sv[cid] = round_sv[i]
                phi[cid] = alpha * phi[cid] + beta * sv[cid]
            time_dict[round_idx] = time.time() - t0
            logging.info("round %d: valuation of %d clients took %.3fs (%d coalition models)", round_idx,
                         len(idxs), time_dict[round_idx], valuer.evaluations)
            w_global = self._finish_round(round_idx, w_locals, res_dict)
            phi_dict[round_idx], sv_dict[round_idx] = list(phi), list(sv)
        self._dump(phi=phi_dict, res=res_dict, sv=sv_dict, client=client_dict, time=time_dict)
        return w_global
