"""Instruction mix of a product kernel's MFMA-carrying basic blocks, counted by class.

    python tools/isa_mix.py [source.hip] [kernel-name-substring] > profiles/r03_attn_isa_mix.txt

Compiles the source for gfx950 exactly as the Makefile does (hipcc -O3, --save-temps into a
temporary directory), finds the kernel's function body in the device assembly and, for every
basic block that issues an MFMA, counts MFMA / VALU (v_exp separately) / LDS / VMEM / s_waitcnt /
s_nop / SALU / branch instructions, plus the most frequent VALU opcodes.  Defaults: the C3
prefill attention, attn_fwd_kernel<48, 4, 1, 64>.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def classify(op: str) -> str:
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_exp"):
        return "v_exp"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "llama3.np_amd/csrc/attention.hip")
    pat = sys.argv[2] if len(sys.argv) > 2 else "_ZN2l315attn_fwd_kernelILi48ELi4ELi1ELi64ELb1EEEvNS_8AttnArgsE"
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "--save-temps", "-c", src, "-o", os.path.join(d, "k.o")], cwd=d, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        asm = [f for f in os.listdir(d) if f.endswith("gfx950.s")][0]
        lines = open(os.path.join(d, asm)).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^\S*" + re.escape(pat) + r"\S*:", l)]
    if not starts:
        sys.exit(f"kernel {pat} not found")
    s0 = starts[0]
    end = next(i for i in range(s0, len(lines)) if lines[i].startswith(".Lfunc_end"))
    name = lines[s0].split(":")[0]
    blocks, cur = [], ["<entry>"]
    for l in lines[s0 + 1:end]:
        if re.match(r"^\.LBB\d+_\d+:", l):
            blocks.append(cur)
            cur = [l.split(":")[0]]
        else:
            cur.append(l)
    blocks.append(cur)
    print(f"# {name}\n# source {os.path.relpath(src, REPO)}; MFMA-carrying basic blocks, static counts")
    tot = collections.Counter()
    for b in blocks:
        c, vc = collections.Counter(), collections.Counter()
        for l in b[1:]:
            t = l.strip()
            if not t or t.startswith((";", ".")):
                continue
            op = t.split()[0]
            k = classify(op)
            c[k] += 1
            if k == "valu":
                vc[op] += 1
        if c["mfma"]:
            tot += c
            per = c["valu"] + c["v_exp"]
            print(f"{b[0]:<14} mfma {c['mfma']:3d} | valu {c['valu']:3d} + v_exp {c['v_exp']:2d} "
                  f"({per / c['mfma']:.2f}/MFMA) | lds {c['lds']:3d} | vmem {c['vmem']:2d} | "
                  f"waitcnt {c['waitcnt']:3d} | nop {c['nop']:2d} | salu {c['salu']:2d} | branch {c['branch']}")
            print(f"{'':14} top VALU: {', '.join(f'{k} {v}' for k, v in vc.most_common(8))}")
    print(f"# total over these blocks: {dict(tot)}")


if __name__ == "__main__":
    main()
