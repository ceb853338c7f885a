"""Summarise a rocprofv3 --kernel-trace --stats run into profiles/ (tracked).

    python tools/rocprof_summary.py gpurun_out/prof/run_kernel_stats.csv profiles/r01_c3 \
        --rows 65536 [--bench gpurun_out/bench.log] [--trace gpurun_out/prof/run_kernel_trace.csv]

Writes <prefix>_kernel_stats.csv (the raw rocprofv3 summary) and <prefix>_summary.md with
per-kernel calls, mean duration and algorithmic TFLOP/s at the stories15M C3 shape.  With
--trace the rows are per (kernel, grid) from the dispatch trace: bench.py's timed forward runs
the batch as two row ranges on concurrent streams (half-size grids, sharing the CUs) and its
roofline pass serialized (full grids, the kernel alone), so the two are reported apart; a
dispatch's rows are --rows x its grid / the kernel's largest grid.
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
        if epi == 1:  # dispatch: 64x96 at K = 288 (O-proj), 128x96 at K = 768 (down); x6 (gemm_x6.h):
            # 4 x 2 waves of 32x48 (O-proj), 4 x 1 waves of 32x96 (down)
            oproj = wn == 2 if "gemm_x6_kernel" in name else tm == 2
            return ("O-proj (+residual)", 2.0 * T * D * D) if oproj else ("down (+residual)", 2.0 * T * FD * D)
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
    ap.add_argument("--trace")
    a = ap.parse_args()
    shutil.copy(a.stats, a.prefix + "_kernel_stats.csv")
    lines = ["| kernel | role | grid | calls | mean µs | algorithmic TFLOP/s | % of peak (fp32 157.3; x6 419.4 fp32-equivalent) |",
             "|---|---|---|---|---|---|---|"]
    rows = []  # (name, grid, calls, mean ns, total ns)
    if a.trace:
        groups = {}
        with open(a.trace) as f:
            for r in csv.DictReader(f):
                g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
                d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                groups.setdefault((r["Kernel_Name"], g), []).append(d)
        for (name, g), ds in groups.items():
            rows.append((name, g, len(ds), sum(ds) / len(ds), sum(ds)))
    else:
        with open(a.stats) as f:
            for r in csv.DictReader(f):
                rows.append((r["Name"], None, int(r["Calls"]), float(r["AverageNs"]), float(r["TotalDurationNs"])))
    gmax = {}
    for name, g, *_ in rows:
        if g:
            gmax[name] = max(gmax.get(name, 0), g)
    for name, g, calls, ns, _ in sorted(rows, key=lambda x: -x[4]):
        t = a.rows * g // gmax[name] if g else a.rows
        role, fl = flops(name, t)
        us = ns / 1e3
        tf = f"{fl / (us * 1e-6) / 1e12:.1f}" if fl else "-"
        peak = 2516.6 / 6 if "gemm_x6_kernel" in name else 157.3  # x6: six bf16 MFMA per fp32 product
        pc = f"{fl / (us * 1e-6) / 1e12 / peak * 100:.1f}" if fl else "-"
        gs = f"{g} ({t} rows)" if g else "-"
        lines.append(f"| `{name[:60]}` | {role} | {gs} | {calls} | {us:.1f} | {tf} | {pc} |")
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
