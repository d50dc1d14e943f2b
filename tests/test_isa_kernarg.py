"""The pooled kernel's launch-parameter re-reads: every instantiation copies the
kernarg segment pointer (s[0:1]) before anything writes s0 / s1, and the production builds spill no
SGPRs (tools/isa_kernarg.py on a hipcc -S listing; CPU only, ~10 s)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.skipif(not shutil.which("hipcc") and not os.path.exists("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_pool_kernel_reads_kernarg_segment_and_spills_no_sgprs(tmp_path):
    from tools import isa_kernarg as K
    listing = str(tmp_path / "pool.s")
    K.compile_pool(listing)
    names = [n for n, _, _ in K.kernels(listing) if "trace_kernel_pool" in n]
    assert len(names) == 8   # (stats, waves per EU 7 / 6, plain / full)
    assert K.check(listing) == []
