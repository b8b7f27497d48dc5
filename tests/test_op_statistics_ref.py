"""``OpStatisticsTest.scala`` ported: Cramér's V on the reference's contingency matrices (2x2, 4x4, 3x6, with empty
rows / columns filtered, an empty matrix), a duplicated noise row lowering Cramér's V, pointwise mutual
information and MI (with the empty-row / -column filter), the empty ``contingencyStats``, max confidences and
supports, and the feature-label correlations agreeing with the full correlation matrix. Matrices are given
column-major as the reference's ``DenseMatrix(rows, cols, values)``."""
import math

import numpy as np
import torch

from transmogrifai_amd.ops import stats as ST
from transmogrifai_amd.stages.preparators.sanity_checker import (_chi2_cramers_v, _filter_empties, _max_conf,
                                                                 _mutual_info, contingency_stats)

TOL = 1e-3


def _dm(rows, cols, vals):
    return np.asarray(vals, np.float64).reshape(cols, rows).T if rows * cols else np.zeros((0, 0))


def _cv(M):
    return _chi2_cramers_v(_filter_empties(M))[0]


def test_cramers_v_2x2():
    assert abs(_cv(_dm(2, 2, [757.0, 726.0, 731.0, 2621.0])) - 0.2921) < TOL


def test_duplicate_noise_row_lowers_cramers_v():
    a = _cv(_dm(3, 2, [100, 0, 50, 0, 100, 50]))
    b = _cv(_dm(4, 2, [100, 0, 50, 50, 0, 100, 50, 50]))
    assert a > b


def test_cramers_v_4x4_and_3x6():
    assert abs(_cv(_dm(4, 4, [5, 15, 20, 68, 29, 54, 84, 119, 14, 14, 17, 26, 16, 10, 94, 7])) - 0.279) < TOL
    assert abs(_cv(_dm(3, 6, [192, 221, 229, 185, 202, 194, 62, 199, 97, 78, 30, 44, 78, 29, 53, 21, 18, 18]))
               - 0.1815) < TOL


def test_cramers_v_filters_empty_rows_and_columns():
    assert math.isnan(_cv(_dm(5, 2, [0.0, 0.0, 0.0, 0.0, 0.0, 5.0, 6.0, 1.0, 2.0, 7.0])))
    assert abs(_cv(_dm(6, 2, [0, 757, 0, 0, 726, 0, 0, 731, 0, 0, 2621, 0])) - 0.2921) < TOL
    assert abs(_cv(_dm(4, 4, [0, 0, 0, 0, 0, 757, 726, 0, 0, 0, 0, 0, 0, 731, 2621, 0])) - 0.2921) < TOL
    assert math.isnan(_cv(_dm(0, 0, [])))


def _pmi(M):
    return _mutual_info(_filter_empties(M))


def _check_pmi(M):
    pmi, mi = _pmi(M)
    expected = {0: [-1.0, 1.5850], 1: [0.2224, -1.5850]}
    assert {int(k) for k in pmi} == set(expected)
    for k, v in pmi.items():
        assert np.allclose(v, expected[int(k)], atol=TOL)
    assert abs(mi - 0.2142) < TOL


def test_pmi_2x2_and_with_empty_rows_and_columns():
    _check_pmi(_dm(2, 2, [10, 15, 70, 5]))
    _check_pmi(_dm(6, 2, [0, 10, 0, 0, 15, 0, 0, 70, 0, 0, 5, 0]))
    _check_pmi(_dm(4, 4, [0, 0, 0, 0, 0, 10, 15, 0, 0, 0, 0, 0, 0, 70, 5, 0]))


def test_pmi_single_label_is_zero():
    pmi, mi = _pmi(_dm(5, 2, [0.0, 0.0, 0.0, 0.0, 0.0, 5.0, 6.0, 1.0, 2.0, 7.0]))
    assert all(x == 0 for v in pmi.values() for x in v)
    assert mi == 0


def test_contingency_stats_of_an_empty_matrix():
    res = contingency_stats(_dm(0, 0, []))
    assert math.isnan(res["cramersV"])
    assert res["pmi"] == {}
    assert math.isnan(res["mutualInfo"])


def test_max_confidences_and_supports():
    conf, sup = _max_conf(_dm(2, 2, [0.0, 500.0, 121.0, 688.0]))
    assert np.allclose(conf, [1.0, 0.5791], atol=TOL) and np.allclose(sup, [0.0924, 0.9076], atol=TOL)
    M = _dm(6, 4, [132.0, 0.0, 189.0, 688.0, 321.0, 0.0, 98.0, 0.0, 823.0, 223.0, 0.0, 366.0,
                   123.0, 14.0, 0.0, 119.0, 0.0, 482.0, 0.0, 0.0, 443.0, 18.0, 321.0, 0.0])
    conf, sup = _max_conf(M)
    assert len(conf) == len(sup) == 6
    assert np.allclose(conf, [0.3739, 1.0, 0.5656, 0.6564, 0.5, 0.5684], atol=TOL)
    assert np.allclose(sup, [0.0810, 0.0032, 0.3337, 0.2404, 0.1472, 0.1945], atol=TOL)


def test_label_correlations_agree_with_the_full_correlation_matrix():
    X = torch.as_tensor(np.random.default_rng(0).standard_normal((100, 100)))
    C = ST.corr_matrix(X)
    full = np.corrcoef(X.numpy(), rowvar=False)[:, -1]
    assert np.allclose(C[:, -1].numpy(), full, rtol=1e-12, atol=0)
