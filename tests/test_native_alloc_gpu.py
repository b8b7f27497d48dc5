"""Grow-only native buffers of the tree growers after a failed growth (ops/csrc/hip/dev_alloc.hpp).

Round 4's 20M-row fault: a buffer that had to grow freed its old block, recorded the new capacity, then the
allocation ran out of memory; the next fit saw ``need <= cap`` and launched on the freed pointer (illegal
address). Here ``tmog_hip_fail_alloc(n)`` makes the n-th native allocation of a growing call fail; that call
must report out of memory, and the next call on the same slot must reallocate and grow exactly the trees a
fresh slot grows (host-planned and device-planned growers)."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.models import tree_engine as te

from test_tree_resident_gpu import _problem


def _grow(pb, resident, slot):
    return te.grow_forest(pb["Xb"], pb["n_bins"], pb["jobs"], mode=te.MODE_GH, kind=te.KIND_NEWTON, t1=pb["t1"],
                          t2=pb["t2"], B=pb["B"], missing_bin=pb["missing_bin"], csr=pb["csr"], collect_leaves=True,
                          groups=1, XbT=pb["Xb"].t().contiguous(), resident=resident, slot_base=slot)


def _forest(f):
    return te.resident_forests([f])[0] if isinstance(f, te.ResidentTree) else f


@pytest.mark.gpu
@pytest.mark.parametrize("resident", [False, True])
@pytest.mark.parametrize("fail_at", [1, 2, 3])
def test_failed_growth_leaves_a_usable_slot(resident, fail_at):
    from transmogrifai_amd.ops import _native
    lib = _native.hip()
    small = _problem("cuda", F=24, n_one=2, N=1500, n_jobs=1, depth=3)
    big = _problem("cuda", F=136, n_one=12, N=40_000, n_jobs=3, depth=7)
    slot = 26 + fail_at                       # a slot no other test uses: starts empty
    ref = _forest(_grow(big, resident, 25))
    _grow(small, resident, slot)              # the slot's buffers at the small size
    lib.tmog_hip_fail_alloc(fail_at)
    try:
        with pytest.raises(RuntimeError, match="out of memory"):
            _grow(big, resident, slot)
    finally:
        lib.tmog_hip_fail_alloc(0)
    torch.cuda.synchronize()                  # the context is healthy: nothing ran on a freed block
    got = _forest(_grow(big, resident, slot))
    for name in ("tree_off", "nodes", "default_left", "value", "gain", "cover"):
        np.testing.assert_array_equal(getattr(ref, name), getattr(got, name), err_msg=name)
    again = _forest(_grow(small, resident, slot))      # and back down: capacity reuse still sound
    np.testing.assert_array_equal(_forest(_grow(small, resident, 25)).nodes, again.nodes)


@pytest.mark.gpu
def test_oom_handler_is_registered():
    from transmogrifai_amd.ops import _native
    _native.hip()
    assert _native._OOM_HANDLER is not None
    _native._release_torch_cache()            # callable from any thread, never raises
