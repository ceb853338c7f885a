"""Where the C3 prefill attention's cycles go: per-wave s_memtime stamps of one launch.

    tools/attn_tune <warm> 1 stamps gpurun_out/attn_stamps.bin   (on the GPU box)
    python tools/attn_stamps.py gpurun_out/attn_stamps.bin

Layout (tools/attn_research.h, ABL & 512): [workgroup][wave][16] uint64 — [0] entry, [1] after
the prologue barrier, [2 + 2t] tile t's compute done, [3 + 2t] after tile t's barrier, [10] exit,
[11] HW_REG_HW_ID, [12] XCC_ID.  Grid of C3: (1, H=6, B=256), 4 waves per workgroup, 4 tiles.
Prints: workgroup lifetime split (prologue, per-tile compute of the busiest wave, barrier wait
per wave, epilogue), per-wave compute per tile against the q-block deal, and how the workgroups
sharing a CU overlap.
"""
import sys
from collections import defaultdict

import numpy as np


def main():
    path = sys.argv[1]
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 4, 16).astype(np.int64)
    n = a.shape[0]
    t0 = a[:, :, 0].min()
    ent, pro, exit_ = a[:, :, 0] - t0, a[:, :, 1] - t0, a[:, :, 10] - t0
    comp = np.stack([a[:, :, 2 + 2 * t] for t in range(4)], -1) - t0   # compute done
    bar = np.stack([a[:, :, 3 + 2 * t] for t in range(4)], -1) - t0    # after barrier
    prev = np.concatenate([pro[:, :, None], bar[:, :, :3]], -1)         # interval start per wave
    work = comp - prev                                                   # compute per tile
    wait = bar - comp                                                    # barrier wait per tile
    life = exit_.max(1) - ent.min(1)
    print(f"workgroups {n}; launch span {(exit_.max() - ent.min()) / 1e3:.1f}k cycles")
    print(f"workgroup lifetime: mean {life.mean() / 1e3:.1f}k cycles")
    pr = (pro.max(1) - ent.min(1))
    print(f"  prologue (entry -> first barrier)   mean {pr.mean():8.0f}  ({pr.mean() / life.mean():5.1%})")
    for t in range(4):
        busiest = work[:, :, t].max(1)
        interval = bar[:, :, t].max(1) - prev[:, :, t].min(1)
        print(f"  tile {t}: interval {interval.mean():8.0f}  busiest wave compute {busiest.mean():8.0f}  "
              f"per-wave compute {np.round(work[:, :, t].mean(0)).astype(int)}  "
              f"per-wave barrier wait {np.round(wait[:, :, t].mean(0)).astype(int)}")
    ep = exit_.max(1) - bar[:, :, 3].max(1)
    print(f"  epilogue (last barrier -> exit)     mean {ep.mean():8.0f}  ({ep.mean() / life.mean():5.1%})")
    tot_work = work.sum(2).mean(0)
    print(f"per-wave total compute {np.round(tot_work).astype(int)} (sum of intervals "
          f"{(bar[:, :, 3].max(1) - pro.min(1)).mean():.0f})")
    # placement: SIMD / CU / SE / XCC, and co-resident workgroups
    hw = a[:, :, 11]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = a[:, :, 12] & 15
    print("wave -> SIMD of the first 6 workgroups:", simd[:6].tolist())
    cu_key = (xcc[:, 0] * 8 + se[:, 0]) * 32 + sh[:, 0] * 16 + cu[:, 0]
    per_cu = defaultdict(list)
    for i in range(n):
        per_cu[int(cu_key[i])].append(i)
    counts = [len(v) for v in per_cu.values()]
    print(f"CUs used {len(per_cu)}, workgroups per CU min {min(counts)} max {max(counts)}")
    # time each CU has >= 1 and 2 workgroups resident
    occ1, occ2, span = [], [], []
    for wgs in per_cu.values():
        ev = []
        for i in wgs:
            ev += [(ent[i].min(), 1), (exit_[i].max(), -1)]
        ev.sort()
        cur, last, o1, o2 = 0, ev[0][0], 0, 0
        for t, d in ev:
            if cur >= 1:
                o1 += t - last
            if cur >= 2:
                o2 += t - last
            cur += d
            last = t
        occ1.append(o1)
        occ2.append(o2)
        span.append(ev[-1][0] - ev[0][0])
    print(f"per CU: span {np.mean(span) / 1e3:.1f}k cycles, >=1 WG resident {np.mean(occ1) / np.mean(span):.1%}, "
          f">=2 WGs resident {np.mean(occ2) / np.mean(span):.1%}")


if __name__ == "__main__":
    main()
