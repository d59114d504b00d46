"""No kernel writes through the scalar data cache (CPU-only check).

Scalar memory stores and atomics, and the scalar cache's write-back /
discard, are not used anywhere in the product's device code: every store
goes through the vector path (global / buffer / LDS).  This test greps the
gfx950 ISA of dist-lr_amd/csrc/dlr_kernels.hip (the `make asm` dump, the
same source the library's code object is built from) for those mnemonics.
It names them, so it is listed in .gpurunignore: no GPU run loads it.
"""
from __future__ import annotations

import os
import subprocess

import pytest

from test_abi import ROOT, _kernel_bodies

FORBIDDEN = ("s_store_", "s_atomic_", "s_buffer_store_", "s_buffer_atomic_", "s_scratch_store",
             "s_dcache_wb", "s_dcache_discard")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_no_scalar_stores_or_atomics():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "dist-lr_amd"), "asm"], check=True)
    with open(os.path.join(ROOT, "dist-lr_amd", "build", "dlr_kernels.s")) as f:
        bodies = _kernel_bodies(f.read())
    assert len(bodies) > 20
    bad = []
    for name, body in bodies.items():
        for line in body:
            op = line.split()[0] if line and not line.startswith((";", ".")) else ""
            if op.startswith(FORBIDDEN):
                bad.append((name[:80], line))
    assert not bad, bad[:10]
