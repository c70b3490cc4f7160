"""Summarise a rocprofv3 rocpd SQLite DB (``-d DIR -o run`` without --output-format csv):
per-kernel totals (top_kernels view) grouped like tools/prof_summary.py, optional CSV dump.
usage: python tools/prof_db_summary.py run_results.db [steps] [out.csv]"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(db.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))


def grp(n):
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        return "hipBLASLt GEMM"
    for key, g in (("grouped_gemm", "moe grouped GEMM"), ("attn_fwd", "attn fwd"), ("attn_bwd_dkdv", "attn bwd dkdv"),
                   ("attn_bwd_dq", "attn bwd dq"), ("adamw", "adamw"), ("xent", "xent"), ("norm_", "norm"),
                   ("colsum", "norm"), ("glu", "glu"), ("rope", "rope"), ("emb_", "embedding"),
                   ("sqsum", "grad-norm"), ("moe_", "moe route/permute"), ("combine", "moe combine"),
                   ("gather_rows", "moe gather"), ("scatter_grad", "moe combine"), ("copyBuffer", "copies"),
                   ("rccl", "rccl"), ("nccl", "rccl")):
        if key in n:
            return g
    return "torch elementwise/other"


g = {}
for name, calls, tot, avg, pct in rows:
    k = grp(name)
    g[k] = g.get(k, 0.0) + float(tot)
T = sum(g.values())
print(f"{'group':32s} {'ms/step':>9s} {'%':>6s}")
for k, v in sorted(g.items(), key=lambda x: -x[1]):
    print(f"{k:32s} {v / 1e3 / steps:9.2f} {v / T * 100:6.1f}")
print(f"{'TOTAL':32s} {T / 1e3 / steps:9.2f}")
if len(sys.argv) > 3:
    with open(sys.argv[3], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
        for r in rows:
            w.writerow([r[0][:200], r[1], round(r[2], 3), round(r[3], 3), round(r[4], 3)])
