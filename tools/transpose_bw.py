"""transpose2d bandwidth and exactness at the headline / Gemma / ViT operand shapes; A/B a build variant by running it
once more with SPA_EXT_SO=ab/_C_<variant>.so (tools/build_variant.sh NAME -DSPA_TRANSPOSE_TS=.. / -DSPA_TRANSPOSE_DIAG=1)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from solvingpapers_amd.ops import _ext
ops = _ext.ops()
for R, C in ((8192, 4096), (4096, 14336), (14336, 4096), (28672, 4096), (50432, 768), (8192, 2048)):
    x = torch.randn(R, C, device="cuda").bfloat16()
    y = ops.transpose2d(x)
    assert torch.equal(y, x.t().contiguous())
    for _ in range(3): ops.transpose2d(x)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20): ops.transpose2d(x)
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    print(f"{os.environ.get('SPA_EXT_SO', 'in-tree'):20s} [{R}, {C}] {ms * 1e3:7.1f} us  {2 * R * C * 2 / ms / 1e9:5.2f} TB/s", flush=True)
