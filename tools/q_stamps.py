#!/usr/bin/env python3
"""Phase timeline of the quaternion reduction from a -DQSTAMPS build
(dwh_debug_qeig writes $QSTAMPS_FILE: per site step j, 16 s_memrealtime
stamps at 100 MHz: [0..7] k_q_rs wave 0, [8..14] k_q_pass workgroup 0).
Prints the mean of each phase (us) over 4 bins of the steps.
Usage: python tools/q_stamps.py stamps.bin"""
import sys

import numpy as np

RS = ["entry->loads", "loads->sum1", "sum1->bar", "bar->colupd", "colupd->sum2", "sum2->stores", "stores"]
PS = ["entry->bar1", "bar1->loop", "loop->bfly", "bfly->bar2", "bar2->Astore", "Astore->part"]


def main():
    st = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 16).astype(np.int64)
    ok = (st[:, 0] > 0) & (st[:, 8] > 0)
    st = st[ok]
    n = len(st)
    d_rs = np.diff(st[:, 0:8], axis=1) * 0.01       # 100 MHz -> us
    d_ps = np.diff(st[:, 8:15], axis=1) * 0.01
    gap_rp = (st[:, 8] - st[:, 7]) * 0.01            # rs last stamp -> pass entry
    gap_pr = (st[1:, 0] - st[:-1, 14]) * 0.01        # pass last stamp -> next rs entry
    bins = np.array_split(np.arange(n), 4)
    print(f"{n} steps; phase means (us) over 4 bins of steps")
    for nm, col in [(f"rs {x}", d_rs[:, i]) for i, x in enumerate(RS)] + [("rs->pass gap", gap_rp)] + \
            [(f"pass {x}", d_ps[:, i]) for i, x in enumerate(PS)]:
        print(f"{nm:24s}" + " ".join(f"{col[b].mean():7.2f}" for b in bins))
    print(f"{'pass->next rs gap':24s}" + " ".join(f"{gap_pr[b[:-1]].mean():7.2f}" for b in bins))
    per = (st[1:, 0] - st[:-1, 0]) * 0.01
    print(f"{'step (rs entry->next)':24s}" + " ".join(f"{per[b[:-1]].mean():7.2f}" for b in bins))


if __name__ == "__main__":
    main()


def clock(path):
    st = np.fromfile(path, dtype=np.uint64).reshape(-1, 16).astype(np.int64)
    st = st[st[:, 15] > 0]
    dr = np.diff(st[:, 7]) * 1e-8
    dc = np.diff(st[:, 15])
    print(f"shader clock over the steps: {np.median(dc / dr) / 1e9:.3f} GHz (median), "
          f"{dc.sum() / dr.sum() / 1e9:.3f} GHz (mean)")


if __name__ == "__main__" and len(sys.argv) > 2:
    clock(sys.argv[1])
