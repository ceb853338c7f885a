"""Weight loading — drop-in for the reference's ``utils.load_parameters``.

Reference: ``utils.py:4-5`` returns ``np.load(model_path)``: a lazy ``NpzFile``
mapping from HF-style tensor names to fp32 arrays stored ``[out, in]``
row-major.  We return the same object (pickle stays disabled, NumPy's
default), so ``weight.get(name)`` and ``weight[name]`` behave identically.

``weight_names`` lists every key the forward pass reads; the device runtime
uses it to fail early on a missing tensor instead of the reference's late
``AttributeError`` on ``None.T`` (``llama3.py:133-136``).
"""

from typing import List

import numpy as np


def load_parameters(model_path):
    return np.load(model_path, allow_pickle=False)


def weight_names(n_layers: int) -> List[str]:
    names = ["model.embed_tokens.weight", "model.norm.weight", "lm_head.weight"]
    for i in range(n_layers):
        p = f"model.layers.{i}."
        names += [
            p + "self_attn.q_proj.weight",
            p + "self_attn.k_proj.weight",
            p + "self_attn.v_proj.weight",
            p + "self_attn.o_proj.weight",
            p + "mlp.gate_proj.weight",
            p + "mlp.up_proj.weight",
            p + "mlp.down_proj.weight",
            p + "input_layernorm.weight",
            p + "post_attention_layernorm.weight",
        ]
    return names
