"""Offline TunableOp tuning of recorded GEMMs, one shape at a time with progress output.

    python tools/tune_gemms.py <untuned.csv> <results.csv>

Reads already-tuned shapes from <results.csv> (skips them), tunes every remaining
``Gemm*`` line of <untuned.csv> over the hipBLASLt + rocBLAS solution sets, and rewrites
<results.csv> after each shape, so an interrupted run keeps its progress.
"""
import os
import sys
import threading
import time

os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1"
os.environ["PYTORCH_TUNABLEOP_RECORD_UNTUNED"] = "0"
os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "15")

import torch  # noqa: E402
import torch.cuda.tunable as tunable  # noqa: E402


def main(untuned, results):
    tunable.enable(True)
    tunable.tuning_enable(True)
    tunable.set_filename(results, False)
    done = set()
    if os.path.exists(results):
        tunable.read_file(results)
        done = {",".join(l.split(",")[:2]) for l in open(results) if l.startswith("Gemm")}
    todo = []
    max_dim = int(os.environ.get("SPA_TUNE_MAX_DIM", "100000"))
    for line in open(untuned):
        if line.startswith(("Gemm", "ScaledGemm")):
            key = ",".join(line.strip().split(",")[:2])
            dims = [int(x) for x in key.split(",")[1].split("_")[1:4]]
            if max(dims) > max_dim:
                print(f"skip (dim > {max_dim}): {key}", flush=True)
                continue
            if key not in done and line not in todo:
                todo.append(line)
    print(f"{len(done)} tuned, {len(todo)} to tune", flush=True)
    for i, line in enumerate(todo):
        t = time.time()
        stop = threading.Event()

        def progress():  # the tuning call is silent for a minute or more per shape
            while not stop.wait(30):
                print(f"    ... tuning {line.strip()}: {time.time() - t:.0f}s", flush=True)
        th = threading.Thread(target=progress, daemon=True)
        th.start()
        tunable._process_single_offline_gemm(line, torch.cuda.current_device())
        torch.cuda.synchronize()
        stop.set()
        th.join()
        _write(results)
        print(f"[{i + 1}/{len(todo)}] {line.strip()}  {time.time() - t:.1f}s", flush=True)


def _write(path):
    """Rewrite the results CSV (validators + every tuned op) from the in-memory database."""
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        for k, v in tunable.get_validators():
            f.write(f"Validator,{k},{v}\n")
        for op, params, sol, ms in tunable.get_results():
            f.write(f"{op},{params},{sol},{ms}\n")
    os.replace(tmp, path)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
