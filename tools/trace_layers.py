"""Per-layer kernel durations from a rocprofv3 --kernel-trace CSV (stories15M, 6 layers).

    python tools/trace_layers.py gpurun_out/prof/run_kernel_trace.csv

Prints, for each GEMM / attention kernel of the C3 forward, the median duration of its
layer-0 launches next to the median of the other layers (layer 0 gathers its input rows
from the embedding table, so its QKV and O-proj launches differ from the rest).
"""
import csv
import statistics
import sys

ROLES = {"QKV": "4, 3, 3, 4", "O-proj": "2, 3, 1, 3", "gate|up": "4, 4, 2, 3", "down": "4, 3, 1, 2",
         "attention": "attn_fwd_kernel"}


def main(path, n_layers=6):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
    for role, tag in ROLES.items():
        d = [t for n, t in seq if tag in n]
        if len(d) < n_layers:
            continue
        first = [t for i, t in enumerate(d) if i % n_layers == 0]
        rest = [t for i, t in enumerate(d) if i % n_layers]
        print(f"{role:10s} launches {len(d):4d}  layer 0 median {statistics.median(first):8.1f} us"
              f"  layers 1..{n_layers - 1} median {statistics.median(rest):8.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
