"""13-qubit tiles (h = 7) on the host: the tile-height switch, the planner's pass counts and the
generated persistent pass kernels ("13-qubit tiles").  No GPU calls."""
import re

import pytest


@pytest.fixture
def tile7(qsim):
    from qsim_amd.plan import set_tile_height
    set_tile_height(7)
    yield
    set_tile_height(-1)


def test_tile_height_switch_bounds(qsim):
    from qsim_amd.plan import set_tile_height
    with pytest.raises(Exception):
        set_tile_height(8)
    set_tile_height(-1)


def test_wider_tiles_never_need_more_passes(qsim):
    from qsim_amd.plan import plan_fused
    for n in (24, 28, 30):
        for seed in (42, 1, 3):
            c = qsim.createRandomHCCircuit(n, 100, seed)
            assert plan_fused(c, 7)[2] <= plan_fused(c, 6)[2], (n, seed)


def test_generated_kernels_are_persistent_at_h7(qsim, tile7):
    from qsim_amd.plan import jit_source
    src = jit_source(qsim.createRandomHCCircuit(30, 100, 42))
    kernels = re.findall(r"__launch_bounds__\((\d+), (\d+)\)\nqk\d+", src)
    # 13-qubit passes, plus passes whose gates fit 12 qubits (mixed heights, QSIM_TILE_MIX)
    assert ("512", "1") in kernels and all(k in (("512", "1"), ("256", "2")) for k in kernels)
    assert "__shared__ double2 tile[8192]" in src
    # multi-stage passes walk their tiles (peeled first tile + loop) and prefetch the next one
    assert "for (;;)" in src and "tile_at(more ? it + 1 : it)" in src


def test_default_height_unchanged(qsim):
    from qsim_amd.plan import jit_source
    src = jit_source(qsim.createRandomHCCircuit(30, 100, 42))
    kernels = re.findall(r"__launch_bounds__\((\d+), (\d+)\)\nqk\d+", src)
    assert kernels and all(k == ("256", "2") for k in kernels)
    assert "for (;;)" not in src
