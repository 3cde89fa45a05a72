"""The d2q9_pf_velocity case of tests/test_kept_fields.py (walls with wetting, a bubble,
the generic perturbation): python tests/pf2_case.py <out.npz> wrote
tests/data/pf2_ref.npz with the model that stored the wall normals every step, pulled
every density in PhaseIter and ran WallIter on every node."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))


def run(device="cpu", steps=6):
    from model_cases import make_case, perturb
    lat = make_case("d2q9_pf_velocity", device, shape=(40, 24, 1))
    lat.init()
    perturb(lat)
    lat.iterate(steps)
    out = {"f": lat.fields_interior().double().cpu().numpy().copy()}
    for g, v in lat.globals.items():
        out["g_" + g] = np.array([v])
    out["PF_q"] = lat.quantity("PhaseField").double().cpu().numpy().copy()
    return out


if __name__ == "__main__":
    np.savez(sys.argv[1], **run())
