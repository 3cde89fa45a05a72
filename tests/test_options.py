"""Option formulas (reference src/models.R:41-66) and the lazily resolved variant table."""
import pytest

from tclb_amd.models import registry
from tclb_amd.models.options import FormulaError, expand, parse


def names(model, formula):
    return [v.name for v in expand(model, formula)]


def test_products_and_autosym_levels():
    assert names("d2q9", "bc*autosym") == ["d2q9_bc", "d2q9_autosym", "d2q9_bc_autosym", "d2q9",
                                           "d2q9_autosym2", "d2q9_bc_autosym2"]
    assert names("x", "") == ["x"]
    assert names("m", "OutFlow") == ["m_OutFlow", "m"]


def test_minus_one_drops_the_plain_model():
    v = names("rd", "(A+B)*(T+E)-1")
    assert "rd" not in v
    assert set(v) == {"rd_A", "rd_B", "rd_T", "rd_E", "rd_A_T", "rd_A_E", "rd_B_T", "rd_B_E"}


def test_interaction_with_parenthesised_sum():
    v = set(names("d3q27_PSM", "MS*KL*TRT*(NEBB+SUP+(NEBB+SEP):singlekernel)"))
    assert len(v) == 40
    assert "d3q27_PSM_SEP" not in v and "d3q27_PSM_SEP_singlekernel" in v
    assert "d3q27_PSM_MS_KL_TRT_NEBB_singlekernel" in v
    assert "d3q27_PSM_NEBB_SUP" not in v


def test_name_order_follows_first_appearance():
    v = names("d3q27_pf_velocity",
              "(q27 + OutFlow  + BGK + thermo*planarBenchmark)*autosym*geometric*staircaseimp*isograd*tprec")
    assert "d3q27_pf_velocity_thermo_planarBenchmark" in v
    assert "d3q27_pf_velocity_thermo_planarBenchmark_autosym2_geometric" in v
    assert "d3q27_pf_velocity_q27_thermo" not in v
    assert len(v) == len(set(v)) == 336


def test_bad_formula():
    with pytest.raises(FormulaError):
        parse("a ** b")


def test_reference_example_models_resolve():
    # model names quoted in the headers of reference example cases
    for n in ("d3q27q27_cm_cht_OutFlowNeumann_AVG_IBB", "d2q9q9_cm_cht_OutFlowNeumann_AVG_IBB",
              "d3q27_cumulant_AVG", "d3q27_cumulant_IB_SMAG", "d2q9_bc_autosym2", "wave2D_autosym",
              "d2q9_reaction_diffusion_system_SIR_ModifiedPeng_Heun"):
        assert registry.variant_status(n) == "ok", n
        m = registry.get(n)
        assert m.name == n


def test_every_default_model_is_a_reference_variant_or_standalone():
    allv = set(registry.all_variants())
    for n in registry.names():
        assert n in allv


def test_every_implemented_variant_builds_a_model():
    ok = [v for v in registry.all_variants() if registry.variant_status(v) == "ok"]
    assert len(ok) > 370
    for v in ok:
        m = registry.get(v)
        assert m.name == v and m.fields


def test_unknown_and_unimplemented_names():
    with pytest.raises(KeyError):
        registry.get("d2q9_nonexistent_option")
    st = registry.variant_status("auto_WMRT_FMT")
    assert st == "ok" or st.startswith("not implemented")


def _wave(model, nx, u0, flags=None, steps=30):
    import numpy as np
    import torch
    from tclb_amd.lattice import Lattice
    lat = Lattice(model, (nx, 4, 1))
    if flags is not None:
        lat.set_flags(np.broadcast_to(flags, (lat.NZ, lat.NY, nx)).copy())
    lat.set_setting("Speed", 0.3)
    lat.set_setting("Viscosity", 0.02)
    lat.init()
    st = lat.fields_interior().clone()
    st[0] = torch.as_tensor(np.broadcast_to(u0, st[0].shape).copy(), dtype=st.dtype)
    lat.set_fields_interior(st)
    lat.iterate(steps)
    return lat.field("u")[0, 0].numpy().copy()


def test_wave2d_autosym_mirrors_the_full_domain():
    """half domain [0, L] with SymmetryX_minus at 0 and SymmetryX_plus at L reproduces the
    periodic full domain of length 2L whose initial state is even about x=0 and x=L"""
    import numpy as np
    L = 12
    xf = np.arange(2 * L)
    u_full0 = np.exp(-0.1 * np.minimum(xf, 2 * L - xf) ** 2)          # even about 0 and L
    full = _wave("wave2D", 2 * L, u_full0)
    from tclb_amd.models import registry
    m = registry.get("wave2D_autosym")
    fl = np.zeros((1, 1, L + 1), dtype=np.uint16)
    fl[..., 0] = m.node_type("SymmetryX_minus").value
    fl[..., L] = m.node_type("SymmetryX_plus").value
    half = _wave("wave2D_autosym", L + 1, u_full0[:L + 1], flags=fl)
    np.testing.assert_allclose(half, full[:L + 1], rtol=0, atol=1e-13)
    assert np.abs(full - u_full0).max() > 1e-3       # the wave actually moved
