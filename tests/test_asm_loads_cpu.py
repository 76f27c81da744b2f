"""The inline-asm load audit (scripts/tools/check_asm_loads.py): a synthetic
assembly listing exercises the walker, and the paged decode's code object -- the pipelined
kernel with hand-counted waits -- must have no compiler access to an in-flight load's registers."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts", "tools"))

import check_asm_loads as cal  # noqa: E402

_LISTING = """_Z1kv:                                ; @_Z1kv
\t;;#ASMSTART
\tglobal_load_dwordx4 v[2:5], v[2:3], off nt
\t;;#ASMEND
\t;;#ASMSTART
\tglobal_load_dwordx4 v[6:9], v[6:7], off nt
\t;;#ASMEND
\tv_mov_b32_e32 v20, v30
\t;;#ASMSTART
\ts_waitcnt vmcnt(1)
\t;;#ASMEND
\tv_add_f32_e32 v21, v2, v3
\t{use6}
\ts_waitcnt vmcnt(0)
\tv_add_f32_e32 v22, v6, v7
\ts_endpgm
"""


def _audit(use6):
    fns = cal.functions(_LISTING.format(use6=use6))
    assert list(fns) == ["_Z1kv"]
    return cal.audit(fns["_Z1kv"])


def test_walker_clean_listing():
    # v[2:5] retired by vmcnt(1) (one younger load), v[6:9] by vmcnt(0): no hazard
    n, hz = _audit("v_mov_b32_e32 v23, v24")
    assert n == 2 and hz == []


def test_walker_flags_copy_before_wait():
    # a copy of v7 while its load is still in flight (only vmcnt(1) so far)
    n, hz = _audit("v_accvgpr_write_b32 a13, v7")
    assert n == 2 and len(hz) == 1
    assert "v[6:9]" in hz[0][2] and "a13" in hz[0][3]


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None and not os.path.exists(
    "/opt/rocm/bin/hipcc"), reason="hipcc not available")
@pytest.mark.timeout(900)
def test_paged_decode_asm_loads_clean():
    asm = cal.device_asm(os.path.join(ROOT, "lumen", "csrc", "kernels", "paged_attention.hip"))
    total, bad = 0, []
    for name, lines in cal.functions(asm).items():
        n, hz = cal.audit(lines)
        total += n
        bad += [(name, h) for h in hz]
    assert total > 0, "no inline-asm loads found: the pipelined kernel was not compiled"
    assert not bad, bad[:3]
