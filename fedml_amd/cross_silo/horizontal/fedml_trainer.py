"""Cross-silo client-side trainer wrapper (reference: `cross_silo/horizontal/fedml_trainer.py:4-72`)."""


class FedMLTrainer:
    def __init__(self, client_index, train_data_local_dict, train_data_local_num_dict, test_data_local_dict,
                 train_data_num, device, args, model_trainer):
        self.trainer = model_trainer
        self.client_index = client_index
        self.train_data_local_dict = train_data_local_dict
        self.train_data_local_num_dict = train_data_local_num_dict
        self.test_data_local_dict = test_data_local_dict
        self.all_train_data_num = train_data_num
        self.device = device
        self.args = args
        self.train_local = None
        self.local_sample_number = None
        self.test_local = None

    def update_model(self, weights):
        self.trainer.set_model_params(weights)

    def update_dataset(self, client_index):
        self.client_index = client_index
        if self.train_data_local_dict is not None:
            self.train_local = self.train_data_local_dict[client_index]
            self.local_sample_number = self.train_data_local_num_dict[client_index]
            self.test_local = (self.test_data_local_dict or {}).get(client_index)
        self.trainer.set_id(client_index)

    def train(self, round_idx=None):
        self.args.round_idx = round_idx
        self.trainer.train(self.train_local, self.device, self.args)
        return self.trainer.get_model_params(), self.local_sample_number

    def test(self):
        tr = self.trainer.test(self.train_local, self.device, self.args)
        te = self.trainer.test(self.test_local, self.device, self.args) if self.test_local is not None else None
        return tr, te
