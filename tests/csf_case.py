"""The d2q9_csf case of tests/test_kept_fields.py: a drop on a wall (wetting angle,
surface tension); python tests/csf_case.py <out.npz> wrote tests/data/csf_ref.npz with
the model that stored the wall normals in every iteration."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def run(steps=6):
    from test_csf import _lat

    def walls(m, lat, fl):
        fl[:, lat.gy:lat.gy + 2, :] = m.node_type("Wall").value
    lat = _lat("d2q9_csf", (32, 24), (16, 5, 5), walls, SurfaceTensionRate=0.01, WettingAngle=0.6)
    lat.iterate(steps)
    out = {"f": lat.fields_interior().double().numpy().copy(),
           "nw_q": lat.quantity("WallNormal").double().numpy().copy()}
    for g, v in lat.globals.items():
        out["g_" + g] = np.array([v])
    return out


if __name__ == "__main__":
    np.savez(sys.argv[1], **run())
