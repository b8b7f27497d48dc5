"""Columnar Parquet ingest (readers/columnar.py) against the generic pandas path (readers/base.py): identical
datasets -- values, null masks, text dictionaries and codes, key -- over several row groups, nulls at row-group
boundaries, float32 / float64 / int columns."""
import numpy as np
import pandas as pd
import pytest
import torch

from transmogrifai_amd.features.builder import FeatureBuilder
from transmogrifai_amd.readers.files import DataReaders


def _frame(n, seed=0):
    rng = np.random.default_rng(seed)
    r32 = rng.standard_normal(n).astype(np.float32)
    r64 = rng.standard_normal(n)
    r64[rng.random(n) < 0.2] = np.nan
    r64[36:38] = np.nan                                   # across the 37-row row-group boundary
    ints = pd.array(rng.integers(-5, 50, n), dtype="Int64")
    ints[rng.random(n) < 0.1] = pd.NA
    cats = np.array(["a", "bb", "", "c d"], dtype=object)[rng.integers(0, 4, n)]
    cats[rng.random(n) < 0.15] = None
    txt = np.array([f"w{k} z" for k in rng.integers(0, 30, n)], dtype=object)
    return pd.DataFrame({"key": [f"k{i}" for i in range(n)], "r32": r32, "r64": r64, "i": ints,
                         "cat": cats, "txt": txt, "y": (rng.random(n) < 0.4).astype(np.float64)})


def _features():
    return [FeatureBuilder.Real("r32").as_predictor(), FeatureBuilder.Real("r64").as_predictor(),
            FeatureBuilder.Integral("i").as_predictor(), FeatureBuilder.PickList("cat").as_predictor(),
            FeatureBuilder.Text("txt").as_predictor(), FeatureBuilder.RealNN("y").as_response()]


def _read(path, dev, columnar, monkeypatch):
    monkeypatch.setenv("TMOG_COLUMNAR", "1" if columnar else "0")
    return DataReaders.Simple.parquet(path, device=dev).generate_dataset(_features())


def _compare(a, b, same_dtype=True):
    assert a.n_rows == b.n_rows and list(a.columns) == list(b.columns)
    assert (a.key is None and b.key is None) or list(a.key) == list(b.key)
    for name in a.columns:
        ca, cb = a[name], b[name]
        if hasattr(ca, "codes"):
            assert ca.vocab == cb.vocab
            assert torch.equal(ca.codes.cpu(), cb.codes.cpu())
        else:
            assert torch.equal(ca.valid.cpu(), cb.valid.cpu()), name
            if same_dtype:
                assert ca.values.dtype == cb.values.dtype
            assert torch.equal(ca.values.cpu().to(torch.float64), cb.values.cpu().to(torch.float64)), name


@pytest.mark.parametrize("rg", [37, 1000])
def test_columnar_parquet_equals_pandas_path_cpu(tmp_path, monkeypatch, rg):
    path = str(tmp_path / "t.parquet")
    _frame(300).to_parquet(path, row_group_size=rg)
    fast = _read(path, "cpu", True, monkeypatch)
    slow = _read(path, "cpu", False, monkeypatch)
    _compare(fast, slow)


def test_columnar_falls_back_for_uncovered_types(tmp_path, monkeypatch):
    from transmogrifai_amd.readers.columnar import parquet_dataset
    path = str(tmp_path / "t.parquet")
    df = _frame(50)
    df["b"] = df["y"] > 0.5
    df.to_parquet(path)
    assert parquet_dataset(path, [FeatureBuilder.Binary("b").as_predictor()], "cpu") is None
    ds = DataReaders.Simple.parquet(path).generate_dataset([FeatureBuilder.Binary("b").as_predictor()])
    assert ds["b"].to_list() == list(df["b"])


@pytest.mark.gpu
def test_columnar_parquet_equals_pandas_path_gpu(tmp_path, monkeypatch):
    path = str(tmp_path / "t.parquet")
    _frame(5000, seed=3).to_parquet(path, row_group_size=777)
    fast = _read(path, "cuda", True, monkeypatch)
    slow = _read(path, "cuda", False, monkeypatch)
    assert fast["r32"].values.dtype == torch.float32 and fast["r32"].values.is_cuda
    _compare(fast, slow, same_dtype=False)


def test_dataset_to_parquet_round_trip(tmp_path, monkeypatch):
    from transmogrifai_amd.readers.columnar import dataset_to_parquet
    path = str(tmp_path / "t.parquet")
    _frame(300, seed=5).to_parquet(path, row_group_size=64)
    ds = _read(path, "cpu", True, monkeypatch)
    out = str(tmp_path / "o.parquet")
    dataset_to_parquet(ds, out, row_group_rows=100)
    monkeypatch.setenv("TMOG_COLUMNAR", "1")
    back = DataReaders.Simple.parquet(out).generate_dataset(_features())
    ds.key = None
    _compare(back, ds)


def _write_nan_table(path, n=500, seed=7):
    """A file whose float columns hold non-null NaNs (written with from_pandas=False: Spark / Arrow writers keep
    NaN apart from null), plus real nulls in another column."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    rng = np.random.default_rng(seed)
    r64 = rng.standard_normal(n)
    r64[rng.random(n) < 0.1] = np.nan
    r32 = rng.standard_normal(n).astype(np.float32)
    r32[5] = np.nan
    nulls = rng.random(n) < 0.2
    rnull = pa.array(np.where(nulls, 0.0, rng.standard_normal(n)), mask=nulls)
    tab = pa.table({"r64": pa.array(r64, from_pandas=False), "r32": pa.array(r32, from_pandas=False),
                    "rnull": rnull, "y": pa.array((rng.random(n) < 0.5).astype(np.float64))})
    assert tab.column("r64").null_count == 0 and tab.column("rnull").null_count > 0
    pq.write_table(tab, path, row_group_size=128)
    return r64, r32


def _nan_features():
    return [FeatureBuilder.Real("r64").as_predictor(), FeatureBuilder.Real("r32").as_predictor(),
            FeatureBuilder.Real("rnull").as_predictor(), FeatureBuilder.RealNN("y").as_response()]


def _check_nan_read(path, dev, monkeypatch, r64, r32):
    monkeypatch.setenv("TMOG_COLUMNAR", "1")
    fast = DataReaders.Simple.parquet(path, device=dev).generate_dataset(_nan_features())
    monkeypatch.setenv("TMOG_COLUMNAR", "0")
    slow = DataReaders.Simple.parquet(path, device=dev).generate_dataset(_nan_features())
    _compare(fast, slow, same_dtype=False)
    assert torch.equal(fast["r64"].valid.cpu(), torch.from_numpy(~np.isnan(r64)))
    assert not bool(torch.isnan(fast["r64"].values).any()) and not bool(torch.isnan(fast["r32"].values).any())
    assert not bool(fast["r32"].valid[5])


def test_columnar_parquet_non_null_nan_is_missing_cpu(tmp_path, monkeypatch):
    path = str(tmp_path / "nan.parquet")
    r64, r32 = _write_nan_table(path)
    _check_nan_read(path, "cpu", monkeypatch, r64, r32)


@pytest.mark.gpu
def test_columnar_parquet_non_null_nan_is_missing_gpu(tmp_path, monkeypatch):
    path = str(tmp_path / "nan.parquet")
    r64, r32 = _write_nan_table(path)
    _check_nan_read(path, "cuda", monkeypatch, r64, r32)


def _csv_read(path, dev, columnar, monkeypatch, **kw):
    monkeypatch.setenv("TMOG_COLUMNAR", "1" if columnar else "0")
    from transmogrifai_amd.readers.files import CSVReader
    return CSVReader(path, device=dev, **kw).generate_dataset(_features())


def test_columnar_csv_equals_pandas_path_cpu(tmp_path, monkeypatch):
    """CSV through pyarrow's parser into the columnar pipeline (readers/columnar.py csv_dataset) gives the
    pandas path's dataset: values, null masks (pandas' NA strings), text dictionaries and codes, key."""
    df = _frame(3000, seed=4)
    path = str(tmp_path / "t.csv")
    df.to_csv(path, index=False, na_rep="")
    from transmogrifai_amd.readers import columnar
    calls = []
    orig = columnar._arrow_dataset
    monkeypatch.setattr(columnar, "_arrow_dataset", lambda *a, **k: calls.append(1) or orig(*a, **k))
    fast = _csv_read(path, "cpu", True, monkeypatch, has_header=True)
    assert calls, "columnar CSV path not taken"
    slow = _csv_read(path, "cpu", False, monkeypatch, has_header=True)
    _compare(fast, slow)


def test_columnar_csv_schema_no_header_and_fallbacks(tmp_path, monkeypatch):
    df = _frame(500, seed=6)
    path = str(tmp_path / "n.csv")
    df.to_csv(path, index=False, header=False, na_rep="NA")
    schema = [("key", "string"), ("r32", "real"), ("r64", "real"), ("i", "integral"), ("cat", "string"),
              ("txt", "string"), ("y", "real")]
    fast = _csv_read(path, "cpu", True, monkeypatch, schema=schema)
    slow = _csv_read(path, "cpu", False, monkeypatch, schema=schema)
    _compare(fast, slow)
    # a junk cell in a numeric column: Arrow cannot parse it, pandas coerces it to missing -> pandas path
    bad = str(tmp_path / "b.csv")
    df2 = df.copy()
    df2["r64"] = df2["r64"].astype(object)
    df2.loc[3, "r64"] = "oops"
    df2.to_csv(bad, index=False)
    from transmogrifai_amd.readers.columnar import csv_dataset
    assert csv_dataset(bad, _features(), "cpu") is None
    ds = _csv_read(bad, "cpu", True, monkeypatch, has_header=True)
    assert not bool(ds["r64"].valid[3])


@pytest.mark.gpu
def test_columnar_csv_equals_pandas_path_gpu(tmp_path, monkeypatch):
    path = str(tmp_path / "g.csv")
    _frame(7000, seed=8).to_csv(path, index=False, na_rep="")
    fast = _csv_read(path, "cuda", True, monkeypatch, has_header=True)
    slow = _csv_read(path, "cuda", False, monkeypatch, has_header=True)
    assert fast["r64"].values.is_cuda
    _compare(fast, slow, same_dtype=False)
