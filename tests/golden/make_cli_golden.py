"""Golden for the reference CLI with its real vocabulary (llama3.py:324-349).

Run in the build container only (needs /root/reference, read-only; nothing of its source is
copied — its vocabulary DATA file and the text its CLI prints are saved):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_cli_golden.py

1. tests/golden/tokenizer.model.np — the reference's vocabulary (a JSON data file, used as-is
   by both CLIs; the GPU box has no /root/reference).
2. tests/golden/cli_dream.json — what `python llama3.py "I have a dream"` of the REFERENCE
   prints (everything before its timing line, and the token count it reports) when run in a
   directory holding that vocabulary and synthetic stories15M weights (the "sharp" preset and
   seed of stories15m_sharp.npz: greedy ids with clear top-1 margins).  The streamed text pins
   the per-token decode, including the reference's `.strip("<s>")` character strip
   (tokenizer.py:65), and the EOS/BOS stop rule (llama3.py:342-343).
"""

import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "llama3.np_amd"))
import synth  # noqa: E402

PROMPT = "I have a dream"


def main():
    vocab = os.path.join(HERE, "tokenizer.model.np")
    shutil.copyfile(os.path.join(REF, "tokenizer.model.np"), vocab)
    g = np.load(os.path.join(HERE, "stories15m_sharp.npz"))
    seed, preset = int(g["seed"]), str(g["preset"])
    w = synth.make_weights(synth.stories15m(1), synth.STORIES15M_HIDDEN, seed=seed, preset=preset)
    assert synth.digest(w) == str(g["weights_sha256"])
    with tempfile.TemporaryDirectory() as d:
        synth.save_npz(os.path.join(d, "stories15M.model.npz"), w)
        os.symlink(vocab, os.path.join(d, "tokenizer.model.np"))
        env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
        out = subprocess.run([sys.executable, os.path.join(REF, "llama3.py"), PROMPT], cwd=d,
                             env=env, check=True, capture_output=True, text=True).stdout
    text, tail = out.split("\n\nToken count: ", 1)
    count = int(tail.split(",", 1)[0])
    res = {"prompt": PROMPT, "seed": seed, "preset": preset, "weights_sha256": str(g["weights_sha256"]),
           "stdout_before_counter": text, "token_count": count,
           "source": "reference llama3.py CLI (llama3.py:324-349) run on these synthetic weights"}
    with open(os.path.join(HERE, "cli_dream.json"), "w", encoding="utf-8") as f:
        json.dump(res, f, indent=1, ensure_ascii=False)
    print(json.dumps({k: v for k, v in res.items() if k != "stdout_before_counter"}))
    print(repr(text[:300]))


if __name__ == "__main__":
    main()
