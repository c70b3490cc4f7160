"""The debug-bounds build of the extension (csrc/include/spa_debug.h) on the GPU:
a child pytest loads ab/_C_dbg.so (built by __graft_entry__.build / tools/build_variant.sh dbg
-DSPA_DEBUG_BOUNDS=1) with SPA_DEBUG_SYNC=1 and runs the ragged-shape cases -- attention at
T = 197/200/300/520 for every head-dim family, the shipped dS-path backward, key split, the short
ViT backward, grouped GEMMs (bf16 + fp8) with empty / odd expert segments, gather / combine, conv,
embedding, cross-entropy -- failing if any device guard fires, plus one deliberate violation that
must be reported (file:line) instead of faulting. One extra process, its output streamed."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
DBG_SO = ROOT / "ab" / "_C_dbg.so"

SELECT = " or ".join([
    "test_flash_attention", "ds_path", "mixed_head_dims", "hd256_variants", "short_bwd", "key_split",
    "grouped_gemm_all_modes", "grouped_gemm8_elementwise", "gemm8_fp8", "fp8_wgrad", "wgrad8_fp8",
    "gather_combine", "permute", "conv_matches_fp32", "test_embedding", "test_xent",
])


@pytest.mark.timeout(900)
def test_debug_bounds_build_runs_ragged_cases_clean():
    if not DBG_SO.exists():
        pytest.skip(f"{DBG_SO} not built (python -c 'import __graft_entry__ as g; g.build()')")
    env = dict(os.environ, SPA_EXT_SO=str(DBG_SO), SPA_DEBUG_SYNC="1")
    cmd = [sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "--timeout", "300",
           "--timeout-method", "thread", str(ROOT / "tests" / "dbg_bounds_child.py"),
           str(ROOT / "tests" / "test_kernels_gpu.py"), str(ROOT / "tests" / "test_moe_gpu.py"),
           str(ROOT / "tests" / "test_conv_gpu.py"), "-k", f"dbg_bounds_child or {SELECT}"]
    rc = subprocess.call(cmd, cwd=ROOT, env=env, timeout=840)
    assert rc == 0, f"debug-bounds child pytest failed (rc={rc})"
