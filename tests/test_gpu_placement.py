"""The snapshot placement probe (csrc/device/snapalloc.hip tclb_snap_probe, Lattice
._alloc_snapshots) for every storage element size: 8 (double), 4 (float, mixed) and 2
(half, half-shift).  The r06q half-shift bench failed in the probe (2-byte elements were
refused); here each size is probed on a small buffer, with fewer planes than the unrolled
widths as well, and the write pass must leave the planes zero."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nf", [27, 19, 5])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32, torch.float16])
def test_snap_probe_every_element_size(dtype, nf):
    from tclb_amd.ops.device import snap_probe_ms
    fs = 1 << 16
    buf = torch.ones(nf * fs, dtype=dtype, device="cuda")
    r, w = snap_probe_ms(buf, nf, fs)
    torch.cuda.synchronize()
    assert r > 0 and w > 0
    assert int(torch.count_nonzero(buf)) == 0          # the write pass zeroed the planes


def test_half_lattice_probes_placement(monkeypatch):
    """a half-shift d3q27 lattice large enough to be probed (threshold lowered) allocates
    its pair through the probe and steps"""
    from tclb_amd.lattice import Lattice
    monkeypatch.setenv("TCLB_PLACE_MIN_GB", "0.01")
    lat = Lattice("d3q27", (64, 64, 64), device=torch.device("cuda", 0), precision="half-shift")
    assert lat.placement is not None and len(lat.placement["kept"]) == 2
    lat.set_setting("nu", 0.05)
    lat.init()
    lat.iterate(2)
    torch.cuda.synchronize()
    assert torch.isfinite(lat.fields_interior().float()).all().item()
