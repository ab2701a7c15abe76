#!/usr/bin/env python3
"""Per-level communication budget of a partitioned wave, from the single-GPU level
trace of the same graph (FGI_TRACE=1 profiles/wave_levels.py <config>: "[fgi] level L push|pull:
frontier F edges T ..." lines; the last wave of the file is used).

For P ranks holding 1-D vertex ranges of N slots (the R-MAT endpoints are scrambled, so a level's
frontier and its targets spread evenly over the ranks):
  push level L  each rank forwards the remote targets its frontier's edges reach, each at most once
                per wave, 4 B each: bytes into one rank <= T_L * (P - 1) / P * 4 / P (every edge of
                the level a distinct remote target: an upper bound), plus the counts all-gather
                (P * (P + 2) * 8 B);
  pull level L  full mode: every rank receives the other ranks' bitmap words, (P - 1) * N / (8 P)
                bytes; delta mode: 8 B per bitmap word that gained a bit since the previous exchange,
                at most min(winners since then, N / 32) words, (P - 1) / P of them from other ranks;
                the engine picks the smaller per level (FGI_OPT_FRONT_EXCHANGE 0).
Time at xGMI: one link per peer pair, LINK_GBS each way; a rank receives from its P - 1 peers in
parallel, so a level's exchange takes (bytes from one peer) / LINK_GBS, plus a fixed per-collective
latency (not modelled: RCCL's small-message latency is tens of microseconds).

Usage: python profiles/comm_budget.py <levels trace (stderr of wave_levels.py)> <n_slots> [P ...]
"""
import re
import sys

LINK_GBS = 153.0   # MI355X_MICROARCH.md / SURVEY.md §5: ~153 GB/s per xGMI link and direction


def last_wave_levels(path):
    waves, cur = [], []
    for line in open(path):
        m = re.match(r"\[fgi\] level (\d+) (push|pull): frontier (\d+) edges (\d+)", line)
        if m:
            lvl = int(m.group(1))
            if lvl == 0 and cur:
                waves.append(cur)
                cur = []
            cur.append((lvl, m.group(2), int(m.group(3)), int(m.group(4))))
    if cur:
        waves.append(cur)
    return [x for x in waves[-1] if x[2] > 0]


def main():
    path, n = sys.argv[1], int(sys.argv[2])
    ps = [int(x) for x in sys.argv[3:]] or [2, 4, 8]
    levels = last_wave_levels(path)
    print(f"| Level | Dir | F | T | " + " | ".join(f"P={p}: bytes in / rank, us at xGMI" for p in ps) + " |")
    print("|---|---|---|---|" + "---|" * len(ps))
    totals = {p: [0.0, 0.0] for p in ps}
    pending = 0   # frontier entries that entered the bitmap since the last exchange (its changed words)
    for lvl, d, f, t in levels:
        pending += f
        cells = []
        for p in ps:
            if d == "push":
                b = t * (p - 1) / p * 4 / p + p * (p + 2) * 8
            else:
                full = (p - 1) * n / (8 * p)
                # winners without rows are not in F: count each changed word twice as a margin
                delta = 8 * min(2 * pending, n / 32) * (p - 1) / p
                b = min(full, delta)
            us = b / max(1, p - 1) / (LINK_GBS * 1e3)
            totals[p][0] += b
            totals[p][1] += us
            cells.append(f"{b / 1e6:.2f} MB, {us:.1f}")
        if d == "pull":
            pending = 0
        print(f"| {lvl} | {d} | {f:,} | {t:,} | " + " | ".join(cells) + " |")
    print("| wave | | | | " + " | ".join(f"{totals[p][0] / 1e6:.1f} MB, {totals[p][1]:.0f}" for p in ps) + " |")


if __name__ == "__main__":
    main()
