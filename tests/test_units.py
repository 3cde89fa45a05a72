import math

import pytest

from tclb_amd.utils.units import UnitEnv, UnitError


def test_basic_parse():
    u = UnitEnv()
    v = u.read_text("0.01m/s")
    assert v.val == pytest.approx(0.01)
    assert list(v.uni[:2]) == [1, -1]
    assert u.read_text("1N").uni[2] == 1  # kg
    assert u.read_text("2mm").val == pytest.approx(2e-3)
    assert u.read_text("1e-3kg/m3").val == pytest.approx(1e-3)
    assert u.read_text("90d").val == pytest.approx(math.pi / 2)
    assert u.read_text("5%").val == pytest.approx(0.05)


def test_gauge_and_alt():
    u = UnitEnv()
    # 1 m = 100 lattice units, 1 s = 1000 iterations, 1 kg/m3 = 1
    u.set_unit("L", u.read_text("1m") / u.read_text("100"), 1)
    u.set_unit("T", u.read_text("1s") / u.read_text("1000"), 1)
    u.set_unit("rho", u.read_text("1kg/m3") / u.read_text("1"), 1)
    u.make_gauge()
    assert u.alt("1m") == pytest.approx(100)
    assert u.alt("1s") == pytest.approx(1000)
    assert u.alt("0.5m/s") == pytest.approx(0.5 * 100 / 1000)
    assert u.alt("1m+2cm") == pytest.approx(102)
    assert u.alt("1e-2m") == pytest.approx(1)
    assert u.alt("3") == 3


def test_underconstructed_gauge_fills_unused():
    u = UnitEnv()
    u.set_unit("L", u.read_text("1m") / u.read_text("10"), 1)
    u.make_gauge()
    assert u.alt("1m") == pytest.approx(10)
    assert u.alt("1s") == pytest.approx(1)


def test_unknown_unit():
    with pytest.raises(UnitError):
        UnitEnv().read_text("1qq")
