"""Register / scratch / LDS budgets of the shipped gfx950 kernels, read from the code object's own metadata
(tools/kernel_resources.py) -- CPU only, no GPU needed.  Guards the residency the measurements assume (DESIGN s.4,
s.5.2a): four solver wavefronts per CU (LDS <= 40 KB each), and the hybrid A* kernel's two wavefronts per SIMD with
its halved scratch (round 6: the lane-coverage test without per-lane interval arrays)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "headland_trajectory_planning_amd", "libhtp.so")


@pytest.fixture(scope="module")
def ks():
    if not os.path.exists(LIB):
        pytest.fail("libhtp.so is not built (python -c 'import __graft_entry__ as g; g.build()')")
    from tools.kernel_resources import kernels
    return kernels(LIB)


def _one(ks, part):
    hits = [v for k, v in ks.items() if part in k]
    assert len(hits) == 1, (part, [k for k in ks if part in k])
    return hits[0]


def test_solver_kernel_fits_four_wavefronts_per_cu(ks):
    r = _one(ks, "obca_solve_kernelILi4ELi4ELi0E")
    assert r["group_segment_fixed_size"] <= 160 * 1024 // 4, r
    assert r["vgpr_count"] <= 512 and r["agpr_count"] <= 256, r   # unified count, of which AGPRs
    assert r["private_segment_fixed_size"] <= 912, r      # round 5's frame; no growth


def test_hastar_kernel_keeps_two_wavefronts_per_simd(ks):
    r = _one(ks, "hastar_kernelILi2E")
    assert r["vgpr_count"] <= 256, r   # .vgpr_count is the unified count (arch + AGPRs): 512 per SIMD lane / 2 waves
    assert r["vgpr_spill_count"] == 0, r
    assert r["private_segment_fixed_size"] <= 528, r       # 1 040 B/lane before the round-6 lane-coverage rewrite


def test_every_kernel_has_metadata(ks):
    names = " ".join(ks)
    for part in ("obca_solve_kernel", "hastar_kernel", "rs_", "ypark", "oge", "classic", "refpath"):
        assert part in names, part
