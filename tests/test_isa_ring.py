"""The EI kernel's asm-load ring is hazard-free in the code the compiler
generated: every spill-free ``gp_score_kernel`` instance in
libmpo.so's gfx950 code objects is checked instruction by instruction by
tests/isa_ring.py -- no instruction reads, writes or copies a VGPR whose
``global_load_dwordx2`` has not been retired by an ``s_waitcnt vmcnt`` on any
control-flow path.  Instances that spill are refused at launch
(``launch_score`` / ``spill_free`` in gp.hip) and are listed, not run.  CPU only."""
import os
import re

import pytest

from tests import isa_ring as R

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi_opt_amd", "libmpo.so")


def test_checker_flags_an_early_read_and_accepts_the_wait():
    ld = [0, "global_load_dwordx2", "v[4:5], v[2:3], off", None]
    use = [12, "v_mfma_f64_16x16x4_f64", "v[20:27], v[8:9], v[4:5], v[20:27]", None]
    end = [16, "s_endpgm", "", None]
    assert R.check_function([ld, use, end])
    wait = [8, "s_waitcnt", "vmcnt(0)", None]
    assert R.check_function([ld, wait, use, end]) == []
    # two loads in flight, vmcnt(1) retires only the older one
    ld2 = [4, "global_load_dwordx2", "v[6:7], v[2:3], off offset:512", None]
    use2 = [12, "v_add_f64", "v[10:11], v[6:7], v[6:7]", None]
    assert R.check_function([ld, ld2, [8, "s_waitcnt", "vmcnt(1)", None], use2, end])
    assert R.check_function([ld, ld2, [8, "s_waitcnt", "vmcnt(1)", None], use, end]) == []
    # a back-edge carrying an outstanding load into a read at the loop head
    loop = [[0, "v_add_f64", "v[10:11], v[4:5], v[4:5]", None],
            [8, "global_load_dwordx2", "v[4:5], v[2:3], off", None],
            [16, "s_cbranch_scc1", "", 0], [20, "s_waitcnt", "vmcnt(0)", None], [24, "s_endpgm", "", None]]
    assert R.check_function(loop)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libmpo.so not built")
def test_gp_score_kernel_ring_is_hazard_free():
    res = {}
    for co in R.gfx950_code_objects(LIB):
        for name, insns in R.functions(R.disassemble(co)).items():
            if "gp_score_kernel" in name:
                spills = any(i[1].startswith("scratch_") for i in insns)
                ring = sum(1 for i in insns if i[1] == "global_load_dwordx2")
                res[name] = (spills, ring, R.check_function(insns))
    assert len(res) >= 48
    groups = {}
    for name, (spills, ring, hazards) in res.items():
        dp, d, occ, md, fin = (int(v) for v in re.findall(r"Li(\d+)E", name.split("gp_score_kernel")[1])[:5])
        groups.setdefault((dp, d, md, fin), []).append((occ, spills, ring, hazards, name))
    for key, variants in groups.items():
        # launch_score runs the highest-occupancy variant that does not spill
        launched = max((v for v in variants if not v[1]), default=None)
        assert launched is not None, key
        for occ, spills, ring, hazards, name in variants:
            if spills:
                continue
            assert ring >= 8, name                   # the ring's loads are present
            assert hazards == [], (name, hazards[:4])
