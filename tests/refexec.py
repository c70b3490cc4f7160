"""Execute the reference notebooks' own PyTorch class/function cells on CPU.

The reference is read-only source; we parse the .ipynb JSON, pick code cells by the
names they define and exec them into a namespace pre-seeded with a small config, so
the parity tests compare our models against the reference's exact code."""
import json
import math
import os
import re

import torch
import torch.nn as nn
import torch.nn.functional as F

REF = os.environ.get("SPA_REFERENCE", "/root/reference")


def available(rel):
    return os.path.exists(os.path.join(REF, rel))


def cells(rel, names):
    nb = json.load(open(os.path.join(REF, rel)))
    out = []
    for c in nb["cells"]:
        if c["cell_type"] != "code":
            continue
        src = "".join(c["source"])
        if any(re.search(rf"^(class|def) {n}\b", src, re.M) for n in names):
            out.append(src)
    return out


def exec_cells(rel, names, ns=None):
    g = {"torch": torch, "nn": nn, "F": F, "math": math}
    g.update(ns or {})
    for src in cells(rel, names):
        exec(compile(src, f"{rel}", "exec"), g)
    return g
