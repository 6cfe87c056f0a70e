"""Host logic of the ECORR path (CPU): the epoch grouping the incremental Metropolis step relies on."""
import numpy as np
import pytest

from pulsar_timing_gibbsspec_amd.ecorr import group_epochs


def test_group_epochs_contiguous_and_stable():
    rng = np.random.default_rng(0)
    ebk = rng.integers(0, 4, 50)
    ecid = 100 + np.arange(50)
    e2, b2, eoff = group_epochs(ecid, ebk, 4)
    assert np.all(np.diff(b2) >= 0)
    assert eoff[0] == 0 and eoff[-1] == 50 and eoff.size == 5
    for k in range(4):
        seg = slice(eoff[k], eoff[k + 1])
        assert np.all(b2[seg] == k)
        assert np.array_equal(e2[seg], ecid[ebk == k])   # stable: the caller's order within a backend
    assert sorted(e2.tolist()) == ecid.tolist()


def test_group_epochs_empty_backend_and_errors():
    e2, b2, eoff = group_epochs([5, 6, 7], [2, 0, 2], 3)
    assert e2.tolist() == [6, 5, 7] and eoff.tolist() == [0, 1, 1, 3]   # backend 1: no epochs
    with pytest.raises(ValueError):
        group_epochs([1, 2], [0], 1)
    with pytest.raises(ValueError):
        group_epochs([1, 2], [0, 3], 2)
