"""Model hyper-parameters — drop-in for the reference's ``config.ModelArgs``.

Reference: ``config.py:5-19`` (``@dataclass ModelArgs``).  Field names, types
and defaults are kept identical so code written against the reference (which
mutates attributes directly, e.g. ``tests/test_llama_implementations.py:46-52``)
keeps working.  Two reference quirks are preserved on purpose:

* ``rope_theta`` is carried but the RoPE tables are always built with base
  10000 (``llama3.py:272-274`` never passes it);
* ``dtype`` is carried but the NumPy reference ignores it in ``llama3.py``.
  The MI355X path always computes in fp32 ("dtype flow").

The helper properties at the bottom are additions used by the device runtime;
they do not change the dataclass's constructor or equality.
"""

from dataclasses import dataclass
from typing import Optional


@dataclass
class ModelArgs:
    # defaults describe Karpathy's stories15M checkpoint (reference README.md:7)
    dim: int = 288
    n_layers: int = 6
    n_heads: int = 6
    n_kv_heads: Optional[int] = None  # None -> n_heads (no GQA)
    vocab_size: int = 32000
    max_seq_len: int = 256
    max_new_tokens: int = 150
    rope_theta: float = 10000.0  # carried, unused (reference quirk)
    norm_eps: float = 1e-6
    max_batch_size: int = 1
    dtype: str = "float32"  # carried, unused by the forward (reference quirk)

    # ---- derived quantities (not dataclass fields) ----
    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    @property
    def kv_heads(self) -> int:
        return self.n_heads if self.n_kv_heads is None else self.n_kv_heads

    @property
    def n_rep(self) -> int:
        return self.n_heads // self.kv_heads
