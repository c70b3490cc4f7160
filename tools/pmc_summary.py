"""Summarise a rocprofv3 --pmc counter_collection.csv: per kernel name, the mean of each counter
over its dispatches, plus VALU/MFMA and LDS/MFMA instruction ratios and MFMA busy share.
    python tools/pmc_summary.py <run_counter_collection.csv> [name-substring ...]"""
import csv
import sys
from collections import defaultdict


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(dict)   # name -> dispatch -> ns (counter rows carry the dispatch's timestamps)
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        if keys and not any(k in name for k in keys):
            continue
        cid = r.get("Dispatch_Id") or r.get("Correlation_Id") or ""
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[name].add(cid)
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            dur[name][cid] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for name, c in sorted(acc.items(), key=lambda x: -x[1].get("SQ_WAVE_CYCLES", 0)):
        n = max(1, len(disp[name]))
        m = {k: v / n for k, v in c.items()}
        line = " ".join(f"{k}={v:.3g}" for k, v in sorted(m.items()))
        print(f"{name[:100]} n={n} {line}")
        mf = m.get("SQ_INSTS_MFMA", 0)
        if mf:
            extra = f"   VALU/MFMA {m.get('SQ_INSTS_VALU', 0) / mf:.2f}  LDS/MFMA {m.get('SQ_INSTS_LDS', 0) / mf:.2f}"
            if m.get("SQ_BUSY_CYCLES"):
                # SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs; SQ_BUSY_CYCLES per SE
                extra += f"  MFMA-busy/SQ-busy {m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / m['SQ_BUSY_CYCLES']:.2f}"
            print(extra)
        if dur[name] and m.get("GRBM_GUI_ACTIVE"):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs: /8 / duration = the clock the dispatch ran at
            # (meaningful for dispatches >> launch overhead, e.g. the 8192^3 hipBLASLt GEMM: 1.87 GHz)
            t = sum(dur[name].values()) / len(dur[name])
            print(f"   mean duration {t / 1e3:.1f} us  clock {m['GRBM_GUI_ACTIVE'] / 8 / t:.2f} GHz")


if __name__ == "__main__":
    main()
