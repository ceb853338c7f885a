"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/pmc_gateup.json <source_hash>
    python tools/pmc_traffic.py gpurun_out/pmc_c5_fetch gpurun_out/pmc_c5_write profiles/pmc_c5_gateup.json <source_hash> c5

(the second form: the Llama-3-shape prefill, bench.py --workload c5, B=64 x L=2048 rows)

<source_hash> is `l3_source_hash()` of the library the passes ran (printed in every bench
line as lib.source_hash); bench.py reports `traffic` only while the library it loads has it.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports exactly half of the
bytes of a wide coalesced streaming read (TCC_EA0_RDREQ x 64 B for 128-B requests), so reads
are doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Both counters are in KiB.
The guide calibrates the x2 only for 16-B-per-lane coalesced streams, so it is applied only to
the kernels whose global reads are that (CALIBRATED: the tiled GEMM's A / W tile loads and the
prefill attention's K / V tile and q loads, and the x6 GEMM's activation / weight-piece tiles (the
same global_load_lds pieces) — whole rows, 16 B per lane, consecutive lanes
consecutive addresses); every other kernel (decode attention: one key row per thread; GEMV /
skinny: lane-split rows; fills and copies) is reported "uncalibrated", as the range
[FETCH + WRITE, 2 x FETCH + WRITE] with no single per-launch figure.
Writes one JSON with the per-launch HBM bytes of every kernel and the headline entry for
the fused gate|up GEMM, which bench.py reports as roofline.traffic.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROWS = 65536
D, FD = 288, 768


def load(d, counter):
    per = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r["Counter_Name"] == counter:
                    per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


CALIBRATED = (r"l3::gemm_lds_kernel<", r"l3::gemm_x6_kernel<", r"l3::attn_fwd_kernel<")


def calibrated(kernel: str) -> bool:
    """Kernels whose global reads are 16-B-per-lane coalesced streams (the access pattern the
    guide's FETCH_SIZE x2 correction is measured on)."""
    return any(c in kernel for c in CALIBRATED)


def main():
    global ROWS, D, FD
    fetch_dir, write_dir, out = sys.argv[1:4]
    c5 = len(sys.argv) > 5 and sys.argv[5] == "c5"
    if c5:
        ROWS, D, FD = 64 * 2048, 4096, 14336
    fe, wr = load(fetch_dir, "FETCH_SIZE"), load(write_dir, "WRITE_SIZE")
    kernels = {}
    for k in fe:
        f_kib = sum(fe[k]) / len(fe[k])
        w_kib = sum(wr.get(k, [0])) / max(1, len(wr.get(k, [0])))
        cal = calibrated(k)
        lo, hi = int((f_kib + w_kib) * 1024), int((2 * f_kib + w_kib) * 1024)
        kernels[k] = {"launches": len(fe[k]), "fetch_kib_raw": round(f_kib, 1),
                      "write_kib": round(w_kib, 1),
                      "fetch_correction": "x2 (16-B/lane coalesced stream)" if cal else "uncalibrated",
                      "hbm_bytes_per_launch": hi if cal else None,
                      "hbm_bytes_range": None if cal else [lo, hi]}
    # the gate|up GEMM is the gemm kernel instantiated with EPI_SWIGLU (5th template argument 2)
    gu = [k for k in kernels if re.search(r"gemm_\w+_kernel<\d+, \d+, \d+, \d+, 2[,>]", k)]
    algo = 4 * (ROWS * D + 2 * FD * D + ROWS * FD)
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes, " +
                     ("python bench.py --workload c5 --layers 2 --steps 1 --warmup 1" if c5 else
                      "python bench.py --steps 2 --warmup 1 --split 1 (every launch full size)"),
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count) for "
                         "the 16-B/lane coalesced streaming kernels only; others uncalibrated (range)",
           "workload_rows": ROWS,
           "source_hash": sys.argv[4],
           "gateup_kernel": gu[0] if gu else None,
           "hbm_bytes_per_launch": kernels[gu[0]]["hbm_bytes_per_launch"] if gu else None,
           "algorithmic_bytes_per_launch": algo,
           "kernels": kernels}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))
    for k, v in kernels.items():
        if v["hbm_bytes_per_launch"] is not None:
            print(f"{v['hbm_bytes_per_launch'] / 1e6:10.1f} MB  {k[:90]}")
        else:
            lo, hi = v["hbm_bytes_range"]
            print(f"{lo / 1e6:6.1f}-{hi / 1e6:.1f} MB (uncalibrated)  {k[:80]}")


if __name__ == "__main__":
    main()
