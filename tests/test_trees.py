

def test_budget_chunks_split_a_batch_that_does_not_fit(monkeypatch):
    """Boosting batches are sized from a device-memory budget up front (models/trees.py _budget_chunks): with a
    budget of 2.5 jobs, 5 jobs run as 3 consecutive chunks; everything fits -> one chunk; CPU -> one chunk."""
    import torch
    from transmogrifai_amd.models import trees as TR
    dev = torch.device("cuda")
    monkeypatch.setattr(torch.cuda, "mem_get_info", lambda d=None: (250, 1000))
    monkeypatch.setattr(torch.cuda, "memory_reserved", lambda d=None: 0)
    monkeypatch.setattr(torch.cuda, "memory_allocated", lambda d=None: 0)
    assert TR._budget_chunks([100] * 5, dev, frac=1.0) == [(0, 2), (2, 4), (4, 5)]
    assert TR._budget_chunks([10] * 5, dev, frac=1.0) == [(0, 5)]
    assert TR._budget_chunks([400, 10], dev, frac=1.0) == [(0, 1), (1, 2)]
    assert TR._budget_chunks([100] * 5, torch.device("cpu")) == [(0, 5)]
    # learner lanes running beside the fit share the free memory: two lanes halve the budget
    from transmogrifai_amd.ops import streams as SP
    SP.set_active_lanes(2)
    try:
        assert TR._budget_chunks([100] * 5, dev, frac=1.0) == [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5)]
    finally:
        SP.set_active_lanes(1)


def test_boost_job_bytes_count_the_level_histograms():
    """A job's estimate grows with its depth and feature count (the grower's two level histograms)."""
    import torch
    from transmogrifai_amd.models import trees as TR
    from transmogrifai_amd.models.base import FitJob
    rows = torch.arange(1_000_000)
    shallow = TR._boost_job_bytes(FitJob({"max_depth": 3}, rows, None), 2_000_000, 100, 32)
    deep = TR._boost_job_bytes(FitJob({"max_depth": 12}, rows, None), 2_000_000, 100, 32)
    assert shallow == 16 * 2_000_000 + 40 * 1_000_000 + 2 * 100 * 33 * 2 * 8 * 4
    assert deep - shallow == 2 * 100 * 33 * 2 * 8 * (2048 - 4)
