"""tools/isa_hazards.py on synthetic gfx950 assembly (CPU): it must flag an
instruction that touches a register an inline-asm load is still filling, and
accept the same code once a counted s_waitcnt retires the load first."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from tools import isa_hazards  # noqa: E402

_HEAD = """\t.text
_Z6kernelv:
"""


def _check(body: str):
    kernels = isa_hazards.parse_kernels((_HEAD + body).splitlines())
    return isa_hazards.check(kernels["_Z6kernelv"])


def test_flags_reuse_of_in_flight_asm_load_register():
    found = _check("""\t;;#ASMSTART
\tglobal_load_dwordx4 v[0:3], v10, s[4:5]
\t;;#ASMEND
\tv_or_b32_e32 v2, s6, v11
\ts_waitcnt vmcnt(0)
\ts_endpgm
""")
    assert found and found[0][1].startswith("v_or_b32") and ("v", 2) in found[0][5]


def test_counted_wait_retires_the_load():
    found = _check("""\t;;#ASMSTART
\tglobal_load_dwordx4 v[0:3], v10, s[4:5]
\t;;#ASMEND
\t;;#ASMSTART
\tglobal_load_dwordx4 v[4:7], v10, s[6:7]
\t;;#ASMEND
\ts_waitcnt vmcnt(1)
\tv_or_b32_e32 v2, s6, v11
\ts_waitcnt vmcnt(0)
\tv_mov_b32_e32 v5, 0
\ts_endpgm
""")
    assert found == []


def test_compiler_loads_and_lds_dma_are_not_tracked():
    # a compiler-issued load gets the compiler's own waits; an LDS-DMA has no
    # register destination
    found = _check("""\tglobal_load_dword v1, v[2:3], off
\t;;#ASMSTART
\ts_mov_b32 m0, s8
\tglobal_load_lds_dwordx4 v12, s[4:5]
\t;;#ASMEND
\tv_add_u32_e32 v1, 1, v1
\tv_mov_b32_e32 v12, 0
\ts_endpgm
""")
    assert found == []


def test_loop_back_edge_carries_in_flight_loads():
    # the load issued at the bottom of the loop is still in flight at the top
    found = _check("""\ts_mov_b32 s0, 4
.LBB0_1:
\tv_mov_b32_e32 v0, 0
\t;;#ASMSTART
\tglobal_load_dwordx4 v[0:3], v10, s[4:5]
\t;;#ASMEND
\ts_sub_u32 s0, s0, 1
\ts_cmp_lg_u32 s0, 0
\ts_cbranch_scc1 .LBB0_1
\ts_waitcnt vmcnt(0)
\ts_endpgm
""")
    assert found and found[0][1].startswith("v_mov_b32_e32 v0")
