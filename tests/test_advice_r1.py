"""ADVICE round-1 fixes: DataBalancer rebalance branching, checkpoint function registry."""
import torch

from transmogrifai_amd.stages import generator as G
from transmogrifai_amd.tuning.splitters import DataBalancer


def test_balancer_up_equal_one_keeps_minority():
    # 7% positives, sampleFraction 0.1: no multiplier fits, getProportions resolves up = 1.0
    n = 100_000
    y = torch.zeros(n, dtype=torch.float64)
    y[:7000] = 1.0
    b = DataBalancer(sample_fraction=0.1, seed=3, max_training_sample=1_000_000)
    s = b.pre_validation_prepare(y)
    assert b.up_fraction == 1.0 and s["upSamplingFraction"] == 1.0
    w = b.weights(torch.arange(n), y)
    assert int((w[:7000] == 1).sum()) == 7000          # every minority row kept exactly once
    assert 0 < int(w[7000:].sum()) < 93000


def test_balancer_up_below_one_samples_without_replacement():
    n = 400_000
    y = torch.zeros(n, dtype=torch.float64)
    y[:30_000] = 1.0
    b = DataBalancer(sample_fraction=0.1, seed=3, max_training_sample=100_000)
    b.pre_validation_prepare(y)
    assert b.up_fraction < 1.0
    w = b.weights(torch.arange(n), y)
    assert int(w.max()) == 1
    kept = int(w[:30_000].sum())
    assert abs(kept - 30_000 * b.up_fraction) < 5 * (30_000 * b.up_fraction) ** 0.5


def test_balancer_already_balanced_reports_zero_up():
    y = torch.tensor([0.0, 1.0] * 500)
    b = DataBalancer(sample_fraction=0.1, seed=1)
    assert b.pre_validation_prepare(y)["upSamplingFraction"] == 0.0


def _secret_fn(r):
    return 1


def test_checkpoint_functions_resolve_only_through_registry():
    assert G.load_extract_fn("os.system") is None
    assert G.load_extract_fn("builtins.eval") is None
    name = G._fn_name(_secret_fn)           # handing a function to a stage registers it
    assert G.load_extract_fn(name) is _secret_fn
    G._FUNCTIONS.pop(name)
    assert G.load_extract_fn(name) is None
    G.register_function(_secret_fn, name="my.extract")
    assert G.load_extract_fn("my.extract") is _secret_fn


def test_pointer_returning_native_functions_declare_pointer_restype():
    """A native function returning a pointer / handle must not default to ctypes' 32-bit int restype
    (a truncated RCCL communicator handle segfaults inside the collective)."""
    import ctypes as C
    import re
    from pathlib import Path
    from transmogrifai_amd.ops import _native as N
    src = Path(N.__file__).parent / "csrc"
    ptr_fns = set()
    for f in list(src.rglob("*.hip")) + list(src.rglob("*.cpp")):
        for m in re.finditer(r"^(?:void|int64_t|size_t|uint64_t)\s*\*?\s*(tmog_\w+)\s*\(", f.read_text(), re.M):
            line = m.group(0)
            if "*" in line or line.startswith(("int64_t", "size_t", "uint64_t")):
                ptr_fns.add(m.group(1))
    declared = set(N._HOST_SIGS) | set(N._HIP_SIGS)
    for fn in sorted(ptr_fns & declared):
        assert N._RESTYPES.get(fn) in (C.c_void_p, C.c_int64, C.c_size_t), fn
