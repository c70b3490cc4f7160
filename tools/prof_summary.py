"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time, grouped."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
def grp(n):
    if n.startswith('Cijk') or n.startswith('Custom_Cijk'): return 'hipBLASLt GEMM'
    if 'attn_fwd' in n: return 'attn fwd'
    if 'attn_bwd_dkdv' in n: return 'attn bwd dkdv'
    if 'attn_bwd_dq' in n: return 'attn bwd dq'
    if 'adamw' in n: return 'adamw'
    if 'xent' in n: return 'xent'
    if 'norm_' in n or 'colsum' in n: return 'norm'
    if 'glu' in n: return 'glu'
    if 'rope' in n: return 'rope'
    if 'emb_' in n or 'cast_kernel' in n: return 'embedding'
    if 'sqsum' in n or 'sum_partials' in n: return 'grad-norm'
    if 'rccl' in n.lower() or 'nccl' in n.lower(): return 'rccl'
    return 'other: ' + n[:60]
g = {}
for r in rows:
    k = grp(r['Name']); g[k] = g.get(k, 0) + float(r['TotalDurationNs'])
print(f"{'group':40s} {'ms/step':>9s} {'%':>6s}")
for k, v in sorted(g.items(), key=lambda x: -x[1]):
    print(f"{k:40s} {v/1e6/steps:9.2f} {v/tot*100:6.1f}")
print(f"{'TOTAL':40s} {tot/1e6/steps:9.2f}")
