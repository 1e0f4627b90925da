"""CPU tests of the feeder data layer: the reference's formats (Armadillo
raw_ascii Dl_new.mat, arma_binary xx.mat), the bundled feeders and the seeded
synthetic feeders / scenario generators."""
import numpy as np
import pytest

from conftest import GOLDEN
from freedm_amd import feeder as F


def test_dl_new_raw_ascii():
    f = F.dl_new_feeder()
    assert f.Dl.shape == (41, 13)
    assert f.n_nodes == 34
    assert np.count_nonzero(f.Dl[:, 0] == 0) == 8          # 8 separator rows
    assert sorted(set(f.Dl[f.Dl[:, 0] != 0, 3].astype(int))) == [1, 2, 3, 4, 5, 7]
    assert f.Z.shape == (21, 3)
    assert f.Dl[0, 4] == pytest.approx(2580 / 5280)          # 800-802 = 2580 ft


def test_xx_mat_arma_binary(tmp_path):
    xx = F.load_arma_bin(f"{GOLDEN}/xx_s1.mat")
    assert xx.shape == (21, 1)
    # the 21 SST Q setpoints: 7 per phase, phases agree to ~1e-14
    a, b, c = xx[0:7, 0], xx[7:14, 0], xx[14:21, 0]
    assert np.allclose(a, b, atol=1e-12) and np.allclose(a, c, atol=1e-12)
    assert xx[0, 0] == pytest.approx(-4.952, abs=1e-3)
    p = tmp_path / "rt.mat"
    F.save_arma_bin(str(p), xx)
    assert open(p, "rb").read() == open(f"{GOLDEN}/xx_s1.mat", "rb").read()
    z = (np.arange(6) + 1j * np.arange(6)[::-1]).reshape(3, 2)
    F.save_arma_bin(str(p), z)
    assert np.array_equal(F.load_arma_bin(str(p)), z)


def test_demo_feeder_integer_division():
    f = F.demo_feeder()
    assert f.Dl.shape == (9, 13) and f.n_nodes == 9
    assert list(f.Dl[[2, 3, 6, 7], 6]) == [-33, 73, 86, -26]      # C++ int division (load_system_data.cpp:32-37)
    assert (f.Dl[5] == 0).all()


def well_formed(Dl):
    seen = {0}
    for m, row in enumerate(Dl):
        if row[0] == 0:
            assert m + 1 < len(Dl) and int(Dl[m + 1, 1]) in seen
            continue
        assert int(row[1]) in seen and int(row[2]) not in seen
        seen.add(int(row[2]))
    return len(seen)


@pytest.mark.parametrize("nn,seed", [(123, 123), (2048, 2048), (300, 7)])
def test_synthetic_feeder_invariants(nn, seed):
    f = F.synthetic_feeder(nn, seed)
    assert f.n_nodes == nn
    assert well_formed(f.Dl) == nn
    assert f.Dl[0, 1] == 0 and f.Dl[0, 2] == 1 and f.Dl[0, 3] == 2
    g = F.synthetic_feeder(nn, seed)
    assert np.array_equal(f.Dl, g.Dl)


def test_scenarios_are_shard_invariant():
    f = F.synthetic_feeder(123, 123)
    all_ = F.scenario_loads(f, np.arange(100))
    part = F.scenario_loads(f, np.arange(37, 61))
    assert np.array_equal(all_[:, :, 37:61], part)
    assert (all_[:, f.Dl[:, 0] == 0, :] == 0).all()
    h = F.hosting_loads(f, np.arange(10))
    assert h.shape == (6, f.nl, 10) and np.isfinite(h).all()
