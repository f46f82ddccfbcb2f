"""SecAgg server aggregator on the HIP engine: the model reconstruction of the reference's
python/fedml/cross_silo/secagg/sa_fedml_aggregator.py:138-184 as ONE ``fa_finite_sum`` launch.

Per key, the reference walks the first-round active clients in order, skipping those whose
upload flag is cleared, reducing mod p after every add (and after taking the first active
client's model when it is flagged), subtracts the aggregate mask, reduces, dequantizes and
multiplies by 1/len(active).  Note that the reference server clears every flag in
``check_whether_all_receive`` (:84-90) before it reconstructs, so in its real message flow only
the first client's model survives; this mirror reproduces whatever the flags say
(tests/golden/g15_*).

The aggregate mask comes from ``aggregate_mask_reconstruction`` (:92-136): BGW decoding of the
secret shares on the host (a few scalars per client), then every surviving client's numpy MT19937
mask stream -- and, for a dropped client, its pairwise streams -- re-expanded ON THE DEVICE and
summed mod p by ``fa_mt_randint_sum`` (bit-exact to numpy's legacy seeding and masked randint;
tests/golden/g21_*).  ``aggregate_model_reconstruction`` keeps that mask on the device.
"""
from __future__ import annotations

import logging
from collections import OrderedDict

import numpy as np
import torch

from ...core.mpc import lightsecagg as fin
from ...core.mpc import secagg as sa
from ...engine import get_engine


class SecAggAggregator(object):
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
        self.flag_client_model_uploaded_dict = dict()
        self.flag_client_ss_uploaded_dict = dict()
        self.num_pk_per_user = 2
        self.targeted_number_active_clients = args.worker_num
        self.privacy_guarantee = int(np.floor(args.worker_num / 2))
        self.prime_number = args.prime_number
        self.precision_parameter = args.precision_parameter
        for idx in range(self.client_num):
            self.flag_client_model_uploaded_dict[idx] = False
            self.flag_client_ss_uploaded_dict[idx] = False
        self.total_dimension = None
        self.dimensions = []
        self._engine = get_engine(None)

    def get_global_model_params(self):
        global_model_params = self.trainer.get_model_params()
        self.dimensions, self.total_dimension = fin.model_dimension(global_model_params)
        return global_model_params

    def set_global_model_params(self, model_parameters):
        self.trainer.set_model_params(model_parameters)

    def add_local_trained_result(self, index, model_params, sample_num):
        logging.info("add_model. index = %d" % index)
        eng = self._engine
        self.model_dict[index] = OrderedDict((k, fin._dev(v, eng, torch.int64)) for k, v in model_params.items())
        self.sample_num_dict[index] = sample_num
        self.flag_client_model_uploaded_dict[index] = True

    def check_whether_all_receive(self):
        for idx in range(self.client_num):
            if not self.flag_client_model_uploaded_dict[idx]:
                return False
        for idx in range(self.client_num):
            self.flag_client_model_uploaded_dict[idx] = False
        return True

    def _aggregate_mask_device(self, active_clients, SS_rx, public_key_list):  # noqa: N803
        """The aggregate mask as an int64 device tensor (see aggregate_mask_reconstruction)."""
        N = self.targeted_number_active_clients
        flags = [self.flag_client_model_uploaded_dict[i] for i in range(N)]
        seeds, signs = sa.mask_streams(N, flags, active_clients, SS_rx, public_key_list, self.privacy_guarantee,
                                       self.prime_number)
        return self._engine.mt_randint_sum(seeds, signs, self.prime_number, self.total_dimension)

    def aggregate_mask_reconstruction(self, active_clients, SS_rx, public_key_list):  # noqa: N803
        """Reference :92-136: for every client i < targeted_number_active_clients, BGW-decode its
        secret from the first T + 1 active clients' shares; a client whose model arrived adds
        randint(0, p, d) seeded by it, a dropped one adds its pairwise masks (sign by index order);
        everything mod p.  Returned as numpy int64 like the reference's."""
        return self._aggregate_mask_device(active_clients, SS_rx, public_key_list).cpu().numpy()

    def aggregate_model_reconstruction(self, active_clients_first_round, active_clients_second_round, SS_rx,
                                       public_key_list):  # noqa: N803
        if type(self).aggregate_mask_reconstruction is SecAggAggregator.aggregate_mask_reconstruction:
            aggregate_mask = self._aggregate_mask_device(active_clients_second_round, SS_rx, public_key_list)
        else:  # a subclass's own mask (kept as the override point it was)
            aggregate_mask = self.aggregate_mask_reconstruction(active_clients_second_round, SS_rx, public_key_list)
        eng = self._engine
        mask = fin._dev(aggregate_mask, eng, torch.int64).reshape(-1)
        p = self.prime_number
        q_bits = self.precision_parameter
        first = active_clients_first_round[0]
        flagged = lambda c: c in self.flag_client_model_uploaded_dict and self.flag_client_model_uploaded_dict[c]  # noqa: E731
        # the running value starts as the first client's own model (averaged_params IS its dict)
        order = [first] + [c for i, c in enumerate(active_clients_first_round) if i > 0 and flagged(c)]
        flags = fin.MOD_EACH | fin.MOD_END | (fin.MOD_FIRST if flagged(first) else 0)
        keys = list(self.model_dict[first].keys())
        segs, masks, pos = [], [], 0
        for j, k in enumerate(keys):
            d = self.dimensions[j]
            col = [self.model_dict[c][k] for c in order]
            if d != col[0].numel():
                raise ValueError(f"cannot reshape array of size {d} into shape {tuple(col[0].shape)}")
            segs.append(col)
            masks.append(mask[pos:pos + d])
            pos += d
        w = 1 / len(active_clients_first_round)
        _, real = eng.finite_sum(segs, p, flags, masks=masks, finite=False, q_bits=q_bits, scale=w)
        averaged_params = OrderedDict()
        for k, r in zip(keys, real):
            averaged_params[k] = r.reshape(1) if r.dim() == 0 else r
        return averaged_params
