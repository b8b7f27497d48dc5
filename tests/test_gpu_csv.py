"""CSV parsed on the GPU (readers/gpu_csv.py, ops/csrc/hip/csv_kernels.hip) against the pyarrow columnar path
(readers/columnar.py csv_dataset): identical float64 / int64 values and validity, identical text codes and
vocabularies -- across chunk boundaries (tiny chunks), quoted fields with separators and escaped quotes, pandas' NA
strings, CRLF line ends, blank lines, a missing final newline and long-mantissa numbers (the host fallback)."""
import numpy as np
import pytest
import torch

from transmogrifai_amd.features import types as T
from transmogrifai_amd.features.builder import FeatureBuilder

pytestmark = pytest.mark.gpu


def _write(path, crlf=False, final_newline=True, n=3000, seed=0):
    rng = np.random.default_rng(seed)
    eol = "\r\n" if crlf else "\n"
    lines = ['"r1","r2","i1","t1","t2"']
    words = ["alpha", "beta", "c,d", 'e""f', "NA", "", "gamma delta", "x"]
    for k in range(n):
        r1 = ["%.9g" % np.float32(rng.normal() * 10.0 ** int(rng.integers(-8, 8))), "", "nan", "-0.0", "1e-30",
              "3.14159265358979323846", "12345678901234567890.5", "7", "-2.5E+3", "NULL"][k % 10]
        r2 = repr(float(rng.normal()))
        i1 = ["1", "", "-42", "9007199254740993", "0"][k % 5]
        t1 = words[rng.integers(0, len(words))]
        t1 = f'"{t1}"' if t1 not in ("", "NA") else t1
        t2 = ["p", "q", "r"][k % 3]
        lines.append(",".join([r1, r2, i1, t1, t2]))
        if k % 997 == 5:
            lines.append("")                      # blank line: skipped
    text = eol.join(lines) + (eol if final_newline else "")
    path.write_bytes(text.encode())


def _features():
    return [FeatureBuilder.Real("r1").as_predictor(), FeatureBuilder.Real("r2").as_predictor(),
            FeatureBuilder.Integral("i1").as_predictor(), FeatureBuilder.Text("t1").as_predictor(),
            FeatureBuilder.PickList("t2").as_predictor()]


@pytest.mark.parametrize("crlf,final_nl,chunk", [(False, True, 1 << 20), (False, False, 4096), (True, True, 7777)])
def test_gpu_csv_matches_arrow(tmp_path, crlf, final_nl, chunk):
    from transmogrifai_amd.readers.columnar import csv_dataset
    from transmogrifai_amd.readers.gpu_csv import gpu_csv_dataset
    p = tmp_path / "d.csv"
    _write(p, crlf, final_nl)
    feats = _features()
    dev = torch.device("cuda")
    ref = csv_dataset(str(p), feats, dev)
    got = gpu_csv_dataset(str(p), feats, dev, chunk_bytes=chunk)
    assert ref is not None and got is not None
    assert got.n_rows == ref.n_rows
    for f in feats:
        a, b = ref[f.name], got[f.name]
        if f.wtype.kind == "text":
            assert list(a.vocab) == list(b.vocab), f.name
            assert torch.equal(a.codes.cpu().to(torch.int32), b.codes.cpu()), f.name
        else:
            va = a.valid.cpu() if a.valid is not None else torch.ones(ref.n_rows, dtype=torch.bool)
            vb = b.valid.cpu() if b.valid is not None else torch.ones(got.n_rows, dtype=torch.bool)
            assert torch.equal(va, vb), f.name
            x, y = a.values.cpu(), b.values.cpu()
            assert x.dtype == y.dtype, f.name
            if x.is_floating_point():
                assert torch.equal(x.view(torch.int64)[va], y.view(torch.int64)[vb]), f.name
            else:
                assert torch.equal(x[va], y[vb]), f.name


def test_ragged_rows_fall_back(tmp_path):
    from transmogrifai_amd.readers.gpu_csv import gpu_csv_dataset
    p = tmp_path / "bad.csv"
    p.write_text('"r1","r2"\n1,2\n3\n')
    assert gpu_csv_dataset(str(p), [FeatureBuilder.Real("r1").as_predictor()], torch.device("cuda")) is None
