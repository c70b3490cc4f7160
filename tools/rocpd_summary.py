"""Per-kernel time summary from a rocprofv3 rocpd SQLite database (--kernel-trace output).

usage: python tools/rocpd_summary.py run_results.db [--top N] [--steps S]
Groups dispatches by a shortened kernel name, prints total ms, share, calls and, with
--steps, ms per step."""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name):
    n = re.sub(r"\(.*$", "", name)
    return n[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--steps", type=int, default=0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    tot = defaultdict(float)
    calls = defaultdict(int)
    for name, dur in c.execute("select name, duration from kernels"):
        k = short(name)
        tot[k] += dur / 1e6
        calls[k] += 1
    all_ms = sum(tot.values())
    print(f"total kernel time {all_ms:.1f} ms over {sum(calls.values())} dispatches")
    print(f"{'ms':>10} {'share':>6} {'calls':>6} {'ms/step':>8}  kernel")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]:
        ps = f"{v / a.steps:8.2f}" if a.steps else "       -"
        print(f"{v:10.2f} {100 * v / all_ms:5.1f}% {calls[k]:6d} {ps}  {k}")


if __name__ == "__main__":
    main()
