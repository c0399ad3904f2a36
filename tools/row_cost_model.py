"""Per-rank statistics of a row-range partition (config 4: 3840 x 2160 x 256,
reference camera), against the measured per-rank frame periods of the
rehearsal (verdict r05 #7: why ranks 3, 4 and 7 take 0.043 ms against
0.036-0.038).  Per range: executed ray-steps (the work the partition
balances), 8x8 tiles with work, the longest ray, the steps of the longest
64-ray tile (a wave's critical path: its lanes march max(n) steps), and the
sum over tiles of max(n) x 64 (lane-slots the range's waves occupy,
idle lanes included).

    python tools/row_cost_model.py [--rows 0,704,...] [--ms 0.0414,...]
"""
import argparse

import numpy as np

import ta_model


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--rows", default="0,704,848,960,1064,1168,1288,1432,2160")
    ap.add_argument("--ms", default="0.0414,0.0375,0.0367,0.0428,0.0429,0.0381,0.0359,0.0430",
                    help="measured per-rank ms per frame (profiles/r05/native_final_c5_c4.txt, 3 streams)")
    a = ap.parse_args()
    ta_model.W, ta_model.H, ta_model.S = a.width, a.height, a.steps
    n, _, _ = ta_model.rays()
    rows = [int(v) for v in a.rows.split(",")]
    ms = [float(v) for v in a.ms.split(",")] if a.ms else [None] * (len(rows) - 1)
    W, H = a.width, a.height
    tn = n[:H - H % 8].reshape(H // 8, 8, W // 8, 8).max(axis=(1, 3))   # per 8x8 tile: its longest ray
    print(f"{W}x{H}x{a.steps}: {int(n.sum())} executed steps; ranges {rows}")
    print("rank  rows  steps(M)  share  tiles_w  max_n  max_tile_n  lane_slots(M)  slot_eff  ms     ms/share")
    tot = n.sum()
    for k in range(len(rows) - 1):
        r0, r1 = rows[k], rows[k + 1]
        s = n[r0:r1].sum()
        t = tn[r0 // 8:r1 // 8]
        slots = (t.astype(np.int64) * 64).sum()
        m = ms[k]
        print(f"{k:4d} {r1 - r0:5d} {s / 1e6:9.2f} {s / tot:6.3f} {int((t > 0).sum()):8d} {int(n[r0:r1].max()):6d} "
              f"{int(t.max()):11d} {slots / 1e6:14.2f} {s / max(slots, 1):9.3f}"
              + (f"  {m:.4f} {m / (s / tot):.4f}" if m else ""))



def makespan_partition(n, parts, b, c, e, W, H):
    """Contiguous ranges on 8-row strips minimising the largest modelled cost
    b * tiles_with_work / 1000 + c * max_n / 100 + e * steps / 1e6 (ms), by a
    binary search on the makespan with a greedy walk (the cost only grows as a
    range extends)."""
    strips = H // 8
    sn = n[:strips * 8].reshape(strips, 8, W // 8, 8)
    tiles = (sn.max(axis=(1, 3)) > 0).sum(1)           # tiles with work per strip
    mx = sn.max(axis=(1, 2, 3))                          # longest ray per strip
    st = sn.sum(axis=(1, 2, 3))

    def walk(T):
        starts, t, m, s = [0], 0, 0, 0
        for k in range(strips):
            t2, m2, s2 = t + tiles[k], max(m, mx[k]), s + st[k]
            if b * t2 / 1e3 + c * m2 / 1e2 + e * s2 / 1e6 > T and k > starts[-1]:
                starts.append(k)
                t2, m2, s2 = tiles[k], mx[k], st[k]
            t, m, s = t2, m2, s2
        return starts

    lo, hi = 0.0, 1.0
    for _ in range(60):
        mid = (lo + hi) / 2
        if len(walk(mid)) <= parts:
            hi = mid
        else:
            lo = mid
    starts = walk(hi)
    while len(starts) < parts:   # split the largest range if the walk used fewer
        starts.append(starts[-1] + 1)
        starts.sort()
    return [8 * s for s in starts] + [H], hi


def candidates():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=8)
    a, _ = ap.parse_known_args()
    ta_model.W, ta_model.H, ta_model.S = 3840, 2160, 256
    n, _, _ = ta_model.rays()
    for b, c, e in [(0.00408, 0.01464, 0.0), (0.00408, 0.01464, 0.0005), (0.003, 0.012, 0.001), (0.005, 0.01, 0.0)]:
        rows, T = makespan_partition(n, a.parts, b, c, e, 3840, 2160)
        print(f"b {b} c {c} e {e}: makespan {T:.4f} ms, rows {','.join(str(v) for v in rows)}")


if __name__ == "__main__":
    import sys
    if "--candidates" in sys.argv:
        sys.argv.remove("--candidates")
        candidates()
    else:
        main()
