"""Host tokenizer — behaviour-identical drop-in for ``tokenizer.Tokenizer``.

Reference: ``tokenizer.py:5-66``.  The file format (``tokenizer.model.np``) is
JSON ``{"tokens": [str]*V, "scores": [float]*V}`` and is used as-is.

Behaviour kept bit-for-bit (north star: "keeping ... tokenizer"):

* characters with no vocabulary entry are silently dropped
  (``tokenizer.py:32-35``, no byte fallback);
* string lookup returns the FIRST index of a duplicated string
  (``list.index`` at ``tokenizer.py:16``; the stories15M vocab has 204
  duplicate strings);
* each round merges the adjacent pair whose merged string has the highest
  score, strictly greater than ``-1e10``; ties go to the leftmost pair
  (``tokenizer.py:36-52``);
* ``decode`` joins the pieces and then strips the *characters* ``<``, ``s``,
  ``/``, ``>`` from both ends (``str.strip`` semantics, ``tokenizer.py:65``),
  so ``decode([471]) == ' wa'``.

What changes is only the cost: ``list.index`` is O(V) per lookup and each
merge round rescans every pair, so the reference is O(n^2 * V).  Here the
first-occurrence index is a dict built once, and a round only re-scores the
two pairs touched by the previous merge (``_pair_score`` cache), giving
O(n^2) worst case with O(1) lookups.
"""

import json
from typing import Dict, List, Optional

_NO_SCORE = -1e10  # reference's initial best score (tokenizer.py:37)


class Tokenizer:
    def __init__(self, model_path: str):
        with open(model_path, encoding="utf-8") as f:
            model = json.load(f)
        self.vocab: List[str] = model["tokens"]
        self.scores: List[float] = model["scores"]
        self.bos_id = 1
        self.eos_id = 2
        first: Dict[str, int] = {}
        for idx, piece in enumerate(self.vocab):
            first.setdefault(piece, idx)  # first duplicate wins, like list.index
        self._first = first

    def str_lookup(self, token: str) -> int:
        return self._first.get(token, -1)

    def _pair_score(self, left: int, right: int):
        merged = self._first.get(self.vocab[left] + self.vocab[right], -1)
        if merged == -1:
            return None
        return self.scores[merged], merged

    def encode(self, text: str, add_bos: bool = True, add_eos: bool = False) -> List[int]:
        ids = [self._first[ch] for ch in text if ch in self._first]
        # pair cache: entry i describes the merge of (ids[i], ids[i+1])
        pairs: List[Optional[tuple]] = [
            self._pair_score(ids[i], ids[i + 1]) for i in range(len(ids) - 1)
        ]
        while True:
            best_at = -1
            best_score = _NO_SCORE
            for i, p in enumerate(pairs):
                if p is not None and p[0] > best_score:  # strict: leftmost tie wins
                    best_score = p[0]
                    best_at = i
            if best_at < 0:
                break
            ids[best_at] = pairs[best_at][1]
            del ids[best_at + 1]
            del pairs[best_at]
            # re-score only the pairs that now touch the merged token
            if best_at > 0:
                pairs[best_at - 1] = self._pair_score(ids[best_at - 1], ids[best_at])
            if best_at < len(ids) - 1:
                pairs[best_at] = self._pair_score(ids[best_at], ids[best_at + 1])
        if add_bos:
            ids.insert(0, self.bos_id)
        if add_eos:
            ids.append(self.eos_id)
        return ids

    def decode(self, ids: List[int]) -> str:
        text = "".join(self.vocab[i] for i in ids)
        return text.strip("<s>").strip("</s>")
