"""The potf2 of the diagonal block broadcasts its pivot column with 64-bit DPP instructions written as inline asm
(gpk_diag_dev.h, potf2_pipelined), which the compiler's hazard recognizer does not see into: every DPP read of a
VGPR must come two wait states after the VALU write of it.  Checked on the built gfx950 code objects."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "gaussianprocessfundamentals_amd", "libgpk.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists(OBJDUMP), reason="libgpk.so or llvm-objdump missing")
def test_no_dpp_read_hazard_in_libgpk():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_dpp_hazard.py"), LIB], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "hazards: 0" in r.stdout
