"""Summarise a rocprofv3 --kernel-trace --stats run into profiles/ (tracked).

    python tools/rocprof_summary.py gpurun_out/prof/run_kernel_stats.csv profiles/r01_c3 \
        --rows 65536 [--bench gpurun_out/bench.log]

Writes <prefix>_kernel_stats.csv (the raw rocprofv3 summary) and <prefix>_summary.md with
per-kernel calls, mean duration and algorithmic TFLOP/s at the stories15M C3 shape.
"""
import argparse
import csv
import json
import re
import shutil

D, FD, H, HD, VS, L = 288, 768, 6, 48, 32000, 256

def flops(name, T):
    """Role and algorithmic FLOPs of a kernel at the C3 shape, from its template arguments."""
    m = re.search(r"gemm_\w+_kernel<(\d+), (\d+), (\d+), (\d+), (\d+)", name)
    if m:
        wm, wn, tm, tn, epi = map(int, m.groups())
        if epi == 2:
            return "gate|up (SwiGLU)", 2.0 * T * D * 2 * FD
        if epi == 3:
            return "QKV (+RMSNorm, RoPE, KV append)", 2.0 * T * D * 3 * D
        if epi == 1:  # dispatch: 64x96 at K = 288 (O-proj), 128x96 at K = 768 (down)
            return ("O-proj (+residual)", 2.0 * T * D * D) if tm == 2 else ("down (+residual)", 2.0 * T * FD * D)
        if epi == 0:
            return "lm_head (+final RMSNorm, last row)", 2.0 * (T // L) * D * VS
    if "attn_fwd_kernel" in name:
        return "causal attention (useful half)", 2.0 * 2 * H * HD * L * (L + 1) / 2 * (T // L)
    return name.split("(")[0], None

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("prefix")
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--bench")
    a = ap.parse_args()
    shutil.copy(a.stats, a.prefix + "_kernel_stats.csv")
    lines = ["| kernel | role | calls | mean µs | algorithmic TFLOP/s | % of 157.3 |", "|---|---|---|---|---|---|"]
    with open(a.stats) as f:
        for r in csv.DictReader(f):
            role, fl = flops(r["Name"], a.rows)
            us = float(r["AverageNs"]) / 1e3
            tf = f"{fl / (us * 1e-6) / 1e12:.1f}" if fl else "-"
            pc = f"{fl / (us * 1e-6) / 1e12 / 157.3 * 100:.1f}" if fl else "-"
            lines.append(f"| `{r['Name'][:60]}` | {role} | {r['Calls']} | {us:.1f} | {tf} | {pc} |")
    if a.bench:
        for line in open(a.bench):
            if line.startswith("{"):
                b = json.loads(line)
                lines += ["", "bench line of the same run:", "", "```", line.strip(), "```"]
                break
    with open(a.prefix + "_summary.md", "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))

if __name__ == "__main__":
    main()
