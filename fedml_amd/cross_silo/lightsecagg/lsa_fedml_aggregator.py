"""LightSecAgg server aggregator on the HIP engine (drop-in for the reference's
python/fedml/cross_silo/lightsecagg/lsa_fedml_aggregator.py, its secure-aggregation part).

The server's two data-parallel steps run on the device:

* ``aggregate_mask_reconstruction`` (reference :101-128): the aggregate mask is LCC-decoded from
  the clients' aggregate encoded masks -- ``fa_lcc_decode`` over the (U x d/(U-T)) buffer, with
  the U x U Lagrange coefficients computed on the host;
* ``aggregate_model_reconstruction`` (reference :130-175): the masked finite models of the
  first-round active clients are summed, the mask is cancelled, the result is reduced mod p,
  dequantized (my_q_inv) and averaged (``* 1/len(active)``) -- ONE ``fa_finite_sum`` launch for
  the whole state_dict.

Client uploads are moved to the device as they arrive (``add_local_trained_result``), so the
reconstruction reads HBM-resident int64 models.  Results are bit-identical to the reference
(tests/golden/g14_*).  Training / evaluation / client selection of the reference class are not
part of this path (scope).
"""
from __future__ import annotations

import logging
from collections import OrderedDict

import numpy as np
import torch

from ...core.mpc import lightsecagg as lsa
from ...engine import get_engine


class LightSecAggAggregator(object):
    def __init__(self, train_global, test_global, all_train_data_num, train_data_local_dict,
                 test_data_local_dict, train_data_local_num_dict, client_num, device, args, model_trainer):
        self.trainer = model_trainer
        self.args = args
        self.train_global = train_global
        self.test_global = test_global
        self.all_train_data_num = all_train_data_num
        self.train_data_local_dict = train_data_local_dict
        self.test_data_local_dict = test_data_local_dict
        self.train_data_local_num_dict = train_data_local_num_dict
        self.client_num = client_num
        self.device = device
        self.model_dict = dict()
        self.sample_num_dict = dict()
        self.aggregate_encoded_mask_dict = dict()
        self.flag_client_model_uploaded_dict = dict()
        self.flag_client_aggregate_encoded_mask_uploaded_dict = dict()
        self.total_dimension = None
        self.dimensions = []
        for idx in range(self.client_num):
            self.flag_client_model_uploaded_dict[idx] = False
            self.flag_client_aggregate_encoded_mask_uploaded_dict[idx] = False
        # the reference fixes U = N and T = floor(N / 2) (lsa_fedml_aggregator.py:58-60)
        self.targeted_number_active_clients = self.client_num
        self.privacy_guarantee = int(np.floor(self.client_num / 2))
        self.prime_number = args.prime_number
        self.precision_parameter = args.precision_parameter
        self._engine = get_engine(None)

    # ------------------------------------------------------------------ model plumbing
    def get_global_model_params(self):
        global_model_params = self.trainer.get_model_params()
        self.dimensions, self.total_dimension = lsa.model_dimension(global_model_params)
        return global_model_params

    def set_global_model_params(self, model_parameters):
        self.trainer.set_model_params(model_parameters)

    def add_local_trained_result(self, index, model_params, sample_num):
        logging.info("add_model. index = %d" % index)
        eng = self._engine
        self.model_dict[index] = OrderedDict((k, lsa._dev(v, eng, torch.int64)) for k, v in model_params.items())
        self.sample_num_dict[index] = sample_num
        self.flag_client_model_uploaded_dict[index] = True

    def add_local_aggregate_encoded_mask(self, index, aggregate_encoded_mask):
        logging.info("add_aggregate_encoded_mask index = %d" % index)
        self.aggregate_encoded_mask_dict[index] = lsa._dev(aggregate_encoded_mask, self._engine, torch.int64)
        self.flag_client_aggregate_encoded_mask_uploaded_dict[index] = True

    def check_whether_all_receive(self):
        for idx in range(self.client_num):
            if not self.flag_client_model_uploaded_dict[idx]:
                return False
        for idx in range(self.client_num):
            self.flag_client_model_uploaded_dict[idx] = False
        return True

    def check_whether_all_aggregate_encoded_mask_receive(self):
        for idx in range(self.client_num):
            if not self.flag_client_aggregate_encoded_mask_uploaded_dict[idx]:
                return False
        for idx in range(self.client_num):
            self.flag_client_aggregate_encoded_mask_uploaded_dict[idx] = False
        return True

    # ------------------------------------------------------------------ secure aggregation
    def aggregate_mask_reconstruction(self, active_clients):
        """Decoded aggregate mask, shape (d', 1) int64 on the device, d' = total dimension rounded
        up to a multiple of U - T (reference :101-128)."""
        d = self.total_dimension
        N = self.client_num
        U = self.targeted_number_active_clients
        T = self.privacy_guarantee
        p = self.prime_number
        d = int(np.ceil(float(d) / (U - T))) * (U - T)
        m = d // (U - T)
        alpha_s = np.array(range(N)) + 1
        beta_s = np.array(range(U)) + (N + 1)
        buf = torch.zeros((U, m), dtype=torch.int64, device=self._engine.device)
        for i, client_idx in enumerate(active_clients):
            buf[i, :] = self.aggregate_encoded_mask_dict[client_idx].reshape(-1)
        eval_points = alpha_s[active_clients]
        flat = lsa.LCC_decoding_with_points(buf, eval_points, beta_s, p, n_out=d)
        return flat.reshape(d, 1)

    def aggregate_model_reconstruction(self, active_clients_first_round, active_clients_second_round):
        aggregate_mask = self.aggregate_mask_reconstruction(active_clients_second_round).reshape(-1)
        p = self.prime_number
        q_bits = self.precision_parameter
        keys = list(self.model_dict[active_clients_first_round[0]].keys())
        segs, masks, shapes = [], [], []
        pos = 0
        for j, k in enumerate(keys):
            col = [self.model_dict[c][k] for c in active_clients_first_round]
            d = self.dimensions[j]
            if d != col[0].numel():
                raise ValueError(f"cannot reshape array of size {d} into shape {tuple(col[0].shape)}")
            segs.append(col)
            masks.append(aggregate_mask[pos:pos + d])
            shapes.append(col[0].shape)
            pos += d
        w = 1 / len(active_clients_first_round)
        _, real = self._engine.finite_sum(segs, p, lsa.MOD_END, masks=masks, finite=False, q_bits=q_bits, scale=w)
        averaged_params = OrderedDict()
        for k, r in zip(keys, real):
            averaged_params[k] = r.reshape(1) if r.dim() == 0 else r  # torch.Tensor([scalar]) for 0-d keys
        self.set_global_model_params(averaged_params)
        return averaged_params
