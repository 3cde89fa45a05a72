"""Objective weights and zonal reads (reference ZoneSettings <global>InObj weights,
src/Lattice.cu.Rt objective accumulation):

- with every <global>InObj weight zero the kernels skip the weighted Objective sum
  (Launch.glob TCLB_GLOB_NOOBJ, core.hpp); the other globals are unchanged;
- zone-dependent weights with zones changing from node to node inside a wavefront: the
  GPU zonal read (core.hpp zonal_read: scalar load for the wave's first zone, vector load
  for the other lanes) equals the CPU executor.
"""
import numpy as np
import pytest
import torch

from conftest import DEVICES
from tclb_amd.lattice import Lattice

N = (32, 16, 8)


def _case(device, weights):
    lat = Lattice("d3q27", N, device=torch.device(device))
    m = lat.model
    zones = [lat.zone_index(f"z{k}") for k in range(3)]
    fl = np.full((lat.NZ, lat.NY, N[0]), m.node_type("MRT").value, dtype=np.uint32)
    x = np.arange(N[0])
    fl |= (np.array(zones)[x % 3] << m.zone_shift)[None, None, :].astype(np.uint32)
    lat.set_flags(fl)
    lat.set_setting("nu", 0.05)
    lat.set_setting("ForceX", 1e-5)
    for k, w in enumerate(weights):
        lat.set_setting("XFluxInObj", w, zone=f"z{k}")
        lat.set_setting("ZFluxInObj", 0.5 * w, zone=f"z{k}")
    lat.init()
    lat.iterate(20)
    lat.iterate(1)
    return lat.globals


@pytest.mark.parametrize("device", DEVICES)
def test_zero_weights_skip_objective(device):
    g0 = _case(device, (0.0, 0.0, 0.0))
    g1 = _case(device, (1.0, 1.0, 1.0))
    assert g0["Objective"] == 0.0
    assert g1["XFlux"] > 0
    assert abs(g1["Objective"] - (g1["XFlux"] + 0.5 * g1["ZFlux"])) <= 1e-12 * abs(g1["XFlux"])
    for k in ("XFlux", "YFlux", "ZFlux"):
        assert g0[k] == g1[k]


@pytest.mark.parametrize("device", DEVICES)
def test_zone_dependent_weights(device):
    """weights 0 / 1 / 3 on zones cycling along x (11, 11 and 10 of the 32 columns): the
    body-forced periodic flow is uniform, so the objective is 41/32 of the x flux"""
    g = _case(device, (0.0, 1.0, 3.0))
    assert abs(g["Objective"] / g["XFlux"] - 41.0 / 32.0) < 1e-9
    if device == "cuda":
        c = _case("cpu", (0.0, 1.0, 3.0))
        for k in ("Objective", "XFlux"):
            assert abs(g[k] - c[k]) <= 1e-11 * abs(c[k])
