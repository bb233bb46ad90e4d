"""gfx950 ring kernels: no s_barrier reached with LDS reads outstanding (tools/lds_barrier_check.py) -- the barrier
guards the slot the next LDS-DMA refills, and gfx950's s_barrier does not wait for a wave's pending ds_reads.
attn_bwd_dq_kernel<64, 3> broke this before round 6 (a sunk MFMA took its operand wait below the barrier), which made
dQ differ run to run.  Compiles attention.hip to device assembly (about 20 s on the CPU)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and shutil.which("hipcc") is None, reason="no hipcc")
def test_attention_barriers_wait_for_lds_reads():
    import lds_barrier_check as chk
    res = chk.scan(chk.device_asm(os.path.join(ROOT, "onetrainer_amd", "csrc", "attention.hip")))
    names = [n for n, _, _ in res]
    assert any("attn_bwd_dq_kernel" in n for n in names) and any("attn_fwd_kernel" in n for n in names), names
    bad = [(n, b) for n, _, b in res if b]
    assert not bad, bad


def test_checker_flags_a_barrier_with_reads_in_flight():
    import lds_barrier_check as chk
    asm = "\n".join(["_Zk:", "ds_read_b128 v[0:3], v4", ".LBB0_1:", "s_barrier", "s_waitcnt lgkmcnt(0)",
                     "s_cbranch_scc1 .LBB0_1", "s_endpgm", ".Lfunc_end0:",
                     "_Zok:", "ds_read_b128 v[0:3], v4", "s_waitcnt lgkmcnt(0)", "s_barrier", "s_endpgm", ".Lfunc_end1:"])
    assert chk.scan(asm) == [("_Zk", 1, 1), ("_Zok", 1, 0)]
