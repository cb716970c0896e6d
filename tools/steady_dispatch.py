"""Steady-state dispatches and kernel time per training iteration from two rocprof summaries
of the same eager bench run at different step counts (tools/profile_bench.sh ... --steps A,
then --steps B; same warm-up): per kernel symbol (calls_B - calls_A) / (B - A), so one-time
work -- first-iteration Adam state and weight packs, capture set-up, the bench's own
fills and copies -- cancels out of the per-iteration figure.

usage: python tools/steady_dispatch.py SUMMARY_A A SUMMARY_B B
"""
import re
import sys


def load(path):
    rows = {}
    for line in open(path):
        m = re.match(r"\s*(\d+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)%\s+(.*)", line)
        if m:
            rows[m.group(5).strip()] = (int(m.group(1)), float(m.group(2)))
    return rows


def main():
    pa, a, pb, b = sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4])
    ra, rb = load(pa), load(pb)
    n = b - a
    out = []
    for k in sorted(set(ra) | set(rb)):
        ca, ta = ra.get(k, (0, 0.0))
        cb, tb = rb.get(k, (0, 0.0))
        out.append(((cb - ca) / n, (tb - ta) / n * 1000.0, k))
    out.sort(key=lambda r: -r[1])
    tot_n = sum(r[0] for r in out)
    tot_us = sum(r[1] for r in out)
    print(f"# steady state per iteration from {pa} ({a} timed steps) and {pb} ({b}): "
          f"{tot_n:.1f} dispatches, {tot_us:.1f} us of kernel time")
    print(f"{'disp/iter':>9} {'us/iter':>9}  kernel")
    for c, us, k in out:
        if abs(c) > 1e-9 or abs(us) > 1e-6:
            print(f"{c:9.2f} {us:9.1f}  {k[:150]}")


if __name__ == "__main__":
    main()
