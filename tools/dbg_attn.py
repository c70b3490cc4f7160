import sys, os, math
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import _ext, reference as R
ops = _ext.ops()
torch.manual_seed(0)
for (T, hd, causal) in [(64, 64, False), (64, 64, True), (128, 128, False), (32, 128, False)]:
    q = torch.randn(1, T, 1, hd, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(1, T, 1, hd, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(1, T, 1, hd, device="cuda", dtype=torch.bfloat16)
    o, lse = ops.attn_fwd(q, k, v, 1 / math.sqrt(hd), causal)
    of, lf = R.attention(q.float(), k.float(), v.float(), causal)
    err = (o.float() - of).abs()[0, :, 0]  # [T, hd]
    lerr = (lse - lf).abs()[0, 0]
    print(f"T{T} hd{hd} causal={causal}: max err {err.max().item():.3f}  lse err {lerr.max().item():.3f}")
    bad_rows = (err.max(1).values > 0.05).nonzero().flatten().tolist()
    bad_cols = (err.max(0).values > 0.05).nonzero().flatten().tolist()
    print("  bad rows", bad_rows[:40]); print("  bad cols", bad_cols[:70])
    badl = (lerr > 0.01).nonzero().flatten().tolist(); print("  bad lse rows", badl[:40])
    # test with v = identity-ish to see key mapping: v[key] = onehot(key % hd)
    if not causal and T <= hd:
        v2 = torch.zeros_like(v); 
        for j in range(T): v2[0, j, 0, j] = 1.0
        q2 = torch.zeros_like(q)  # uniform attention -> o[d] = 1/T for d<T
        o2, _ = ops.attn_fwd(q2, k, v2, 1.0, False)
        print("  uniform probe row0:", (o2[0, 0, 0, :T].float() * T).round().tolist())
