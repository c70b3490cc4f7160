"""Per-kernel-group summary of two rocprofv3 counter passes over a training step:
    python tools/pmc_step_summary.py <pass-a counter_collection.csv> <pass-b counter_collection.csv>
pass a: SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE
pass b: FETCH_SIZE WRITE_SIZE (KB)
Prints, per group, the dispatch time (GRBM_GUI_ACTIVE / 8 XCDs at the measured clock is not
needed: the kernel-trace durations are used), MFMA-busy cycles per SQ-busy cycle, and the HBM
bytes per dispatch."""
import csv
import sys
from collections import defaultdict


def group(n):
    if n.startswith(("Cijk", "Custom_Cijk")):
        return "hipBLASLt GEMM"
    for key, g in (("attn_fwd", "attention fwd"), ("attn_bwd_dq", "attention dQ"), ("attn_bwd_dkdv", "attention dK/dV"),
                   ("adamw", "AdamW"), ("glu", "SwiGLU"), ("norm_", "RMSNorm"), ("rope", "RoPE"), ("xent", "LM-head CE"),
                   ("transpose", "wgrad transposes"), ("emb_", "embedding"), ("sqsum", "grad norm")):
        if key in n:
            return g
    return "other"


def load(path):
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        names[d] = r.get("Kernel_Name", "")
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    return per, names


def main():
    a, na = load(sys.argv[1])
    b, nb = load(sys.argv[2])
    ga = defaultdict(lambda: defaultdict(float))
    for d, c in a.items():
        g = group(na[d])
        ga[g]["n"] += 1
        for k, v in c.items():
            ga[g][k] += v
    gb = defaultdict(lambda: defaultdict(float))
    for d, c in b.items():
        g = group(nb[d])
        gb[g]["n"] += 1
        for k, v in c.items():
            gb[g][k] += v
    print(f"{'group':20s} {'disp':>6s} {'MFMA-busy/SQ-busy':>18s} {'HBM read MB/disp':>17s} {'write MB/disp':>14s}")
    for g in sorted(ga, key=lambda x: -ga[x].get("SQ_BUSY_CYCLES", 0)):
        c = ga[g]
        ratio = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1.0, c.get("SQ_BUSY_CYCLES", 0))
        nbd = max(1.0, gb[g].get("n", 0))
        print(f"{g:20s} {int(c['n']):6d} {ratio:18.2f} {gb[g].get('FETCH_SIZE', 0) / 1024 / nbd:17.1f} "
              f"{gb[g].get('WRITE_SIZE', 0) / 1024 / nbd:14.1f}")


if __name__ == "__main__":
    main()
