"""Host tokenizer parity against the reference's own outputs (CPU).

Fixture: tests/golden/tokenizer.json, produced by the reference Tokenizer.
The vocabulary is the reference's own data file, committed as
tests/golden/tokenizer.model.np (tests/golden/make_cli_golden.py copies it), so
the tests run anywhere, the GPU box included.
"""

import json
import os

import pytest

from conftest import GOLDEN
from tokenizer import Tokenizer

VOCAB = os.path.join(GOLDEN, "tokenizer.model.np")
needs_vocab = pytest.mark.skipif(not os.path.exists(VOCAB), reason="vocab fixture absent")


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(GOLDEN, "tokenizer.json"), encoding="utf-8") as f:
        return json.load(f)


@needs_vocab
def test_encode_matches_reference(fx):
    tok = Tokenizer(VOCAB)
    for case in fx["encode"]:
        assert tok.encode(case["text"]) == case["ids"], case["text"]
        assert tok.encode(case["text"], add_bos=False, add_eos=True) == case["ids_eos"]


@needs_vocab
def test_decode_matches_reference(fx):
    tok = Tokenizer(VOCAB)
    for case in fx["decode"]:
        assert tok.decode(case["ids"]) == case["text"], case["ids"]


@needs_vocab
def test_known_answers():
    tok = Tokenizer(VOCAB)
    assert tok.encode("I have a dream") == [1, 76, 505, 263, 12561]
    assert tok.encode("Once upon a time") == [1, 26222, 2501, 263, 931]
    assert tok.decode([471]) == " wa"  # str.strip("<s>") strips the characters
    assert (tok.bos_id, tok.eos_id) == (1, 2)
    assert tok.str_lookup("<s>") == 1 and tok.str_lookup("no-such-piece") == -1
