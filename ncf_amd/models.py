"""NCF model: the reference's constructor, attribute schema, state_dict keys and
initialisation, with the forward/backward of HIP-resident models routed through
libncf_hip.so.

Mirrors reference ``src/ncf/models.py``:
  * ``__init__``               models.py:5-36  (same submodules, same creation order,
                                                hence the same CPU-generator draws)
  * ``_init_weight``           models.py:38-46
  * ``load_pretrain_weights``  models.py:48-95 (same key mapping, messages, errors)
  * ``forward``                models.py:97-118 -- on a HIP device this is the fused
                               gather/GMF/MFMA-tower kernel (``ncf_amd.ops``); there is
                               no silent fallback to ATen ops on the GPU.  On a CPU
                               device the module evaluates with stock torch CPU ops,
                               i.e. it behaves like the reference module it replaces.
"""
from __future__ import annotations

import torch
import torch.nn as nn


class NCF(nn.Module):
    def __init__(self, user_num, item_num, factor_num, num_layers, dropout, model_type):
        super().__init__()
        self.model_type = model_type
        self.dropout = dropout
        self.factor_num = factor_num
        self.num_layers = num_layers
        self.user_num = user_num
        self.item_num = item_num

        self.embed_user_GMF = nn.Embedding(user_num, factor_num)
        self.embed_item_GMF = nn.Embedding(item_num, factor_num)
        mlp_dim = factor_num * (2 ** (num_layers - 1))
        self.embed_user_MLP = nn.Embedding(user_num, mlp_dim)
        self.embed_item_MLP = nn.Embedding(item_num, mlp_dim)

        modules = []
        width = factor_num * (2 ** num_layers)
        for _ in range(num_layers):
            modules.append(nn.Dropout(p=self.dropout))
            modules.append(nn.Linear(width, width // 2))
            modules.append(nn.ReLU())
            width //= 2
        self.MLP_layers = nn.Sequential(*modules)

        predict_size = factor_num if self.model_type in ["GMF", "MLP"] else factor_num * 2
        self.predict_layer = nn.Linear(predict_size, 1)
        self._init_weight()

    def _init_weight(self):
        nn.init.normal_(self.embed_user_GMF.weight, std=0.01)
        nn.init.normal_(self.embed_item_GMF.weight, std=0.01)
        nn.init.normal_(self.embed_user_MLP.weight, std=0.01)
        nn.init.normal_(self.embed_item_MLP.weight, std=0.01)
        for m in self.MLP_layers:
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
        nn.init.kaiming_uniform_(self.predict_layer.weight, a=1, nonlinearity="sigmoid")

    # ------------------------------------------------------------------ helpers
    def linear_layers(self):
        return [m for m in self.MLP_layers if isinstance(m, nn.Linear)]

    def ordered_params(self):
        """Parameters in flat-buffer / state_dict order."""
        out = [self.embed_user_GMF.weight, self.embed_item_GMF.weight,
               self.embed_user_MLP.weight, self.embed_item_MLP.weight]
        for lin in self.linear_layers():
            out += [lin.weight, lin.bias]
        out += [self.predict_layer.weight, self.predict_layer.bias]
        return out

    def state_dict(self, *args, **kwargs):
        # Parameters of a HIP-resident model are views into one flat buffer
        # (ncf_amd.ops.ensure_flat); hand out standalone tensors so a saved file
        # holds exactly the reference's tensors and nothing else.
        sd = super().state_dict(*args, **kwargs)
        for k, v in list(sd.items()):
            if isinstance(v, torch.Tensor) and getattr(self, "_ncf_flat", None) is not None \
                    and v.untyped_storage().data_ptr() == self._ncf_flat.untyped_storage().data_ptr():
                sd[k] = v.detach().clone()
        return sd

    def load_pretrain_weights(self, gmf_state, mlp_state):
        """Load pretrained GMF and MLP weights for NeuMF-pre (models.py:48-95)."""
        if self.model_type != "NeuMF-pre":
            return
        try:
            self.embed_user_GMF.weight.data.copy_(gmf_state["embed_user_GMF.weight"])
            self.embed_item_GMF.weight.data.copy_(gmf_state["embed_item_GMF.weight"])
            print("    GMF weights loaded successfully")
            self.embed_user_MLP.weight.data.copy_(mlp_state["embed_user_MLP.weight"])
            self.embed_item_MLP.weight.data.copy_(mlp_state["embed_item_MLP.weight"])
            print("    MLP embedding weights loaded successfully")
            n = 0
            for i, layer in enumerate(self.MLP_layers):
                if isinstance(layer, nn.Linear):
                    wk, bk = f"MLP_layers.{i}.weight", f"MLP_layers.{i}.bias"
                    if wk in mlp_state and bk in mlp_state:
                        layer.weight.data.copy_(mlp_state[wk])
                        layer.bias.data.copy_(mlp_state[bk])
                        print(f"    Loaded MLP layer {n} weights")
                    else:
                        print(f"    Warning: Could not find weights for MLP layer {n}")
                        nn.init.xavier_uniform_(layer.weight)
                        if layer.bias is not None:
                            nn.init.zeros_(layer.bias)
                    n += 1
            nn.init.kaiming_uniform_(self.predict_layer.weight, a=1, nonlinearity="sigmoid")
            if self.predict_layer.bias is not None:
                nn.init.zeros_(self.predict_layer.bias)
            print("    NeuMF prediction layer initialized")
        except Exception as e:  # same reporting contract as the reference
            print(f"    Error loading pretrained weights: {e}")
            print("    Available keys in GMF state:", list(gmf_state.keys())[:5])
            print("    Available keys in MLP state:", list(mlp_state.keys())[:5])
            raise RuntimeError(f"Failed to load pretrained weights: {e}")

    # ------------------------------------------------------------------ forward
    def forward(self, user, item):
        if self.embed_user_GMF.weight.is_cuda:
            from . import ops
            return ops.ncf_forward(self, user, item)  # dropout: ops._dropout_layout
        return self._forward_cpu(user, item)

    def _forward_cpu(self, user, item):
        if self.model_type == "GMF":
            output = self.embed_user_GMF(user) * self.embed_item_GMF(item)
        elif self.model_type == "MLP":
            concat = torch.cat((self.embed_user_MLP(user), self.embed_item_MLP(item)), -1)
            output = self.MLP_layers(concat)
        else:
            gmf = self.embed_user_GMF(user) * self.embed_item_GMF(item)
            mlp = self.MLP_layers(torch.cat((self.embed_user_MLP(user), self.embed_item_MLP(item)), -1))
            output = torch.cat((gmf, mlp), -1)
        return self.predict_layer(output).view(-1)
