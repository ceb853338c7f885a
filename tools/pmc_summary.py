"""Aggregate rocprofv3 --pmc counter_collection CSVs per kernel and print derived ratios.

    python tools/pmc_summary.py gpurun_out/pmcA gpurun_out/pmcB [--filter attn]

SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~ SQ_WAVE_CYCLES (MI355X_MICROARCH.md,
rocprofv3 PMC slots); SQ_* cycle counters count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES counts
cycles; SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = extra LDS cycles from conflicts.
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def load(dirs):
    per = defaultdict(lambda: defaultdict(float))
    n = defaultdict(lambda: defaultdict(int))
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for r in csv.DictReader(f):
                    k = r["Kernel_Name"]
                    per[k][r["Counter_Name"]] += float(r["Counter_Value"])
                    n[k][r["Counter_Name"]] += 1
    # mean per dispatch
    return {k: {c: v / n[k][c] for c, v in cs.items()} for k, cs in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    for k, c in sorted(load(a.dirs).items()):
        if a.filter not in k or "rocclr" in k:
            continue
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        line = [k[:70]]
        for name in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                     "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if name in c:
                line.append(f"{name[3:]}/wave {c[name] / wc:.2f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            # per-SIMD MFMA busy vs GPU-active cycles (256 CUs x 4 SIMDs; GRBM summed over 8 XCDs)
            util = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8)
            line.append(f"MFMA busy {util:.2f}")
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            line.append(f"LDS conflict {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:.3f}")
        for name in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
            if name in c:
                line.append(f"{name[9:]} {c[name]:.3g}")
        print(" | ".join(line))


if __name__ == "__main__":
    main()
