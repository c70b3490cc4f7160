"""Summarise a rocprofv3 rocpd database (ROCm 7.2 default output, ``run_results.db``).

Per kernel: calls, total / mean device ms, share; per queue: busy ms; the span from the first
kernel start to the last kernel end and the sum of kernel time (busy union per queue shows
whether two streams' kernels ran side by side).

  python tools/rocpd_summary.py gpurun_out/<dir>/run_results.db [--top 25] [--grep attn]
      [--timeline START_MS:DUR_MS [--merged]] [--comm stream_copy] [--last-step adamw]

--timeline prints every kernel of that window (ms from the first kernel) per stream, with the
idle gaps; --comm NAME reports how much of the time kernels matching NAME (a collective or its
stand-in) ran with / without a concurrent compute kernel on another stream.
"""
from __future__ import annotations

import argparse
import glob
import sqlite3
import sys


def _tab(con, prefix):
    for (name,) in con.execute("select name from sqlite_master where type='table'"):
        if name.startswith(prefix + "_"):
            return name
    raise KeyError(prefix)


def load(path):
    con = sqlite3.connect(path)
    kd, ks = _tab(con, "rocpd_kernel_dispatch"), _tab(con, "rocpd_info_kernel_symbol")
    rows = con.execute(f"select d.start, d.end, d.queue_id, d.stream_id, s.display_name, s.kernel_name "
                       f"from {kd} d join {ks} s on d.kernel_id = s.id").fetchall()
    return rows


def _union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def summarise(rows, top=25, grep=None, out=sys.stdout):
    if grep:
        rows = [r for r in rows if grep in (r[4] or r[5])]
    if not rows:
        print("no kernels", file=out)
        return
    agg = {}
    for s, e, q, st, disp, name in rows:
        k = (disp or name)[:110]
        a = agg.setdefault(k, [0, 0])
        a[0] += 1
        a[1] += e - s
    total = sum(v[1] for v in agg.values())
    span = max(r[1] for r in rows) - min(r[0] for r in rows)
    print(f"kernels {len(rows)}  kernel-time {total / 1e6:.3f} ms  span {span / 1e6:.3f} ms  "
          f"busy-union {_union([(r[0], r[1]) for r in rows]) / 1e6:.3f} ms", file=out)
    byq = {}
    for s, e, q, st, *_ in rows:
        byq.setdefault((q, st), []).append((s, e))
    for (q, st), iv in sorted(byq.items()):
        print(f"  queue {q} stream {st}: {len(iv)} kernels, busy {_union(iv) / 1e6:.3f} ms", file=out)
    print(f"{'ms':>10} {'%':>6} {'calls':>6}  kernel", file=out)
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{t / 1e6:10.3f} {100 * t / total:6.2f} {n:6d}  {k}", file=out)


def _short(name):
    n = name.split("(")[0]
    for pre in ("void ", "spa::"):
        n = n.replace(pre, "")
    return n[:48]


def timeline(rows, start_ms, dur_ms, out=sys.stdout, merged=False):
    """Kernels of the window [start, start + dur) ms from the first kernel (a negative start:
    from the last kernel's end), per stream with idle gaps, or (merged) all streams in start order."""
    t0 = min(r[0] for r in rows)
    if start_ms < 0:
        start_ms += (max(r[1] for r in rows) - t0) / 1e6
    lo, hi = t0 + start_ms * 1e6, t0 + (start_ms + dur_ms) * 1e6
    byq = {}
    for s, e, q, st, disp, name in sorted(rows):
        if e >= lo and s <= hi:
            byq.setdefault((q, st), []).append((s, e, disp or name))
    if merged:
        ev = sorted((s, e, key, n) for key, ks in byq.items() for s, e, n in ks)
        for s, e, key, n in ev:
            print(f"  {(s - t0) / 1e6:9.3f} ms  +{(e - s) / 1e3:8.1f} us  s{key[1]}  {_short(n)}", file=out)
        return
    for key, ks in sorted(byq.items()):
        print(f"-- queue {key[0]} stream {key[1]}", file=out)
        prev = None
        for s, e, n in ks:
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            print(f"  {(s - t0) / 1e6:9.3f} ms  +{(e - s) / 1e3:8.1f} us  gap {gap:7.1f} us  {_short(n)}", file=out)
            prev = e


def comm_overlap(rows, pat, out=sys.stdout):
    comm = [(s, e, st) for s, e, q, st, d, n in rows if pat in (d or n)]
    comp = [(s, e, st) for s, e, q, st, d, n in rows if pat not in (d or n)]
    if not comm:
        print(f"no kernels matching {pat}", file=out)
        return
    comp.sort()
    tot = over = 0
    for cs, ce, cst in comm:
        tot += ce - cs
        iv = [(max(s, cs), min(e, ce)) for s, e, st in comp if e > cs and s < ce and st != cst]
        over += _union(iv) if iv else 0
    print(f"comm kernels '{pat}': {len(comm)}, {tot / 1e6:.3f} ms; with concurrent compute {over / 1e6:.3f} ms "
          f"({100 * over / max(tot, 1):.1f} %)", file=out)


def last_step(rows, pat):
    marks = sorted(r for r in rows if pat in (r[4] or r[5]))
    ends, prev = [], None
    for r in marks:
        if prev is not None and r[0] - prev > 50e6:
            ends.append(prev)
        prev = r[1]
    ends.append(prev)
    if len(ends) < 2:
        return rows
    lo, hi = ends[-2], ends[-1]
    return [r for r in rows if r[0] >= lo and r[1] <= hi]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db", nargs="+")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--grep", default=None)
    ap.add_argument("--timeline", default=None, help="START_MS:DUR_MS (negative START: from the end)")
    ap.add_argument("--merged", action="store_true", help="timeline: all streams in one start-ordered list")
    ap.add_argument("--comm", default=None, help="kernel-name substring of the collective kernels")
    ap.add_argument("--last-step", default=None, metavar="KERNEL",
                    help="summarise only the last training step: the window between the last two "
                         "bursts of KERNEL (e.g. adamw), bursts split at gaps > 50 ms")
    a = ap.parse_args()
    for pat in a.db:
        for path in sorted(glob.glob(pat)):
            print(f"== {path}")
            rows = load(path)
            if a.last_step:
                rows = last_step(rows, a.last_step)
            summarise(rows, a.top, a.grep)
            if a.comm:
                comm_overlap(rows, a.comm)
            if a.timeline:
                st, du = (float(x) for x in a.timeline.split(":"))
                timeline(rows, st, du, merged=a.merged)


if __name__ == "__main__":
    main()
