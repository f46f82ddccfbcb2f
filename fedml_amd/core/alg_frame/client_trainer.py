"""ClientTrainer plugin surface (reference: python/fedml/core/alg_frame/client_trainer.py:7-62).

The trainer-side counterpart of ServerAggregator: a client produces ``(num_samples, state_dict)``
-- the exact input format of the aggregation engine (``get_model_params`` returns a state_dict,
cf. ml/trainer/my_model_trainer_classification.py:15-16 in the reference).  Local DP and data
poisoning hooks (core/dp, core/security) are outside this engine and stay off.
"""
from __future__ import annotations

from abc import ABC, abstractmethod


class ClientTrainer(ABC):
    def __init__(self, model, args):
        self.model = model
        self.id = 0
        self.args = args
        self.local_train_dataset = None
        self.local_test_dataset = None
        self.local_sample_number = 0
        for flag in ("enable_dp", "enable_attack"):
            if getattr(args, flag, False):
                raise NotImplementedError(f"args.{flag}=True is outside the MI355X aggregation engine")

    def set_id(self, trainer_id):
        self.id = trainer_id

    def is_main_process(self):
        return True

    def update_dataset(self, local_train_dataset, local_test_dataset, local_sample_number):
        self.local_train_dataset = local_train_dataset
        self.local_test_dataset = local_test_dataset
        self.local_sample_number = local_sample_number

    @abstractmethod
    def get_model_params(self):
        ...

    @abstractmethod
    def set_model_params(self, model_parameters):
        ...

    def on_before_local_training(self, train_data, device, args):
        pass

    @abstractmethod
    def train(self, train_data, device, args):
        ...

    def on_after_local_training(self, train_data, device, args):
        pass

    def test(self, test_data, device, args):
        pass
