"""Generic per-model set-up used by the catalog-wide tests (CPU smoke + HIP-vs-CPU)."""
import numpy as np
import torch

from tclb_amd.lattice import Lattice
from tclb_amd.models import registry

SMALL_2D = (40, 24, 1)
SMALL_3D = (24, 12, 10)


def collision_value(m, name=None):
    """the node type every node is flagged with: the case's "_flag" (a collision type the
    model's Run() dispatches) or the model's first COLLISION type"""
    flag = case_settings(name or m.name).get("_flag")
    if flag and m.node_type(flag) is not None:
        return m.node_type(flag).value
    for g in ("COLLISION",):
        for n in m.node_types:
            if n.group == g:
                return n.value
    return 0


# model-family settings for a physically meaningful small case (defaults of some models,
# e.g. zero densities of the phase-field models, are not runnable as they stand)
CASE_SETTINGS = {
    "d2q9_npe_guo": {"epsilon": 50.0, "nu": 0.1, "n_inf_0": 1.0, "n_inf_1": 1.0, "el": 1.0, "el_kbT": 1.0,
                     "psi_bc": 0.01},
    "d2q9_poison_boltzmann": {"tau_psi": 1.0, "dt": 1.0, "epsilon": 1.0, "n_inf": 0.02, "z": 1.0, "el": 1.0,
                              "kb": 1.0, "T": 1.0, "psi_bc": 0.01, "psi0": 0.0},
    "d2q9_kuper": {"Density": 1.0, "Temperature": 0.65, "Magic": 0.005, "FAcc": 1.0, "nu": 0.1666},
    "d3q19_kuper": {"Density": 1.0, "Temperature": 0.65, "Magic": 0.005, "FAcc": 1.0, "nu": 0.1666},
    "d3q27_kl": {"eta1": 0.05, "eta2": 0.01, "sigmaY": 1e-5, "m": 1e3, "Lambda": 0.25},
    "d3q27_viscoplastic": {"YieldStress": 1e-4, "nu": 0.1},
    "d2q9_optimalMixing": {"Temperature": 1.0, "MovingWallVelocity": 0.01},
    "sw": {"Height": 1.0, "Gravity": 0.1},
    "d2q9_solid": {"nu": 0.1, "FluidAlfa": 0.1, "SoluteDiffusion": 0.05, "Temperature": 1.0, "Concentration": 0.5,
                   "LiquidusSlope": -1.0, "PartitionCoef": 0.5, "C0": 0.5, "Teq": 1.0},
    "d2q9_kuper_adj": {"InitDensity": 1.0, "WallDensity": 1.0, "Temperature": 0.65, "Magic": 0.005, "FAcc": 1.0,
                       "nu": 0.1666, "MagicA": -0.152, "MagicF": 1.0},
    "d2q9_lee": {"LiquidDensity": 1.0, "VaporDensity": 0.1, "Beta": 0.01, "Kappa": 0.0162, "InitDensity": 0.5,
                 "WallDensity": 0.5},
    "d2q9_pp_LBL": {"T": 0.32, "Density": 0.5},
    "d2q9_pp_MCMP": {"Gc": 1.0, "Density": 1.0, "Density_dry": 0.1},
    "d2q9_pf_pressureEvolution": {"Density_h": 1.0, "Density_l": 0.1, "sigma": 1e-3, "PhaseField": 1.0,
                                  "Radius": 5.0, "CenterX": 20.0, "CenterY": 12.0, "BubbleType": -1.0},
    "d2q9_pf_velocity": {"Density_h": 1.0, "Density_l": 0.1, "sigma": 1e-3, "PhaseField_init": 1.0, "Radius": 5.0,
                         "CenterX": 20.0, "CenterY": 12.0, "BubbleType": -1.0, "bulk_visc": 0.1666},
    "d2q9_reaction_diffusion_system_SIR_ModifiedPeng": {"Init_N": 1.0, "Init_S": 0.9, "Init_I": 0.1,
                                                        "Beta": 0.3, "Beta_w": 0.2, "Gamma": 0.1},
    "d2q9_scmp": {"Kupershtokh_K": 0.009, "Temperature": 0.8, "Density": 1.2, "nu_l": 0.1666, "nu_v": 0.1666,
                  "density_l": 3.0, "density_v": 0.1, "nubuffer": 0.1},
    # no wall plane: the generic perturbation would break the exact -999 wall marker of phi
    "d2q9_csf": {"_no_walls": True, "PhaseField": -0.45, "Mobility": 0.05, "WettingAngle": 0.5, "IntWidth": 0.25, "SurfaceTensionRate": 0.01,
                 "VelocityX": 0.01, "ViscosityStepWidth": 1.0},
    "d3q27_pf_velocity_thermo": {"Density_h": 1.0, "Density_l": 0.1, "sigma": 1e-3, "Viscosity_l": 0.05,
                                 "Viscosity_h": 0.05, "M": 0.05, "PhaseField": 1.0, "Radius": 4.0,
                                 "CenterX": 12.0, "CenterY": 6.0, "CenterZ": 5.0, "BubbleType": -1.0,
                                 "T_init": 1.0, "dT": 0.05, "sigma_T": -1e-4, "k_h": 0.05, "k_l": 0.02,
                                 "cp_h": 1.0, "cp_l": 1.0},
    "d3q27_tePSM_per": {"omegaF": 1.0, "FluidConductivity": 0.2, "SolidConductivity": 0.5},
    # the finite-difference PDEs: their defaults (zero diffusivity, zero velocity) leave a
    # state unchanged, so a benchmark of them would time a copy
    "diffusion2D": {"diff_coeff": 0.1},
    "advection_diffusion2D": {"diff_coeff": 0.1, "ux": 0.05, "uy": 0.02},
    # Run() has no case for the first COLLISION type (CM): flag the higher-order CM collision
    "d2q9q9_cm_cht": {"_flag": "CM_HIGHER"},
    "d3q27_pf_velocity": {"Density_h": 1.0, "Density_l": 0.1, "sigma": 1e-3, "Viscosity_l": 0.05,
                          "Viscosity_h": 0.05, "M": 0.05, "PhaseField": 1.0, "Radius": 4.0,
                          "CenterX": 12.0, "CenterY": 6.0, "CenterZ": 5.0, "BubbleType": -1.0},
}


def case_settings(name):
    if name in CASE_SETTINGS:
        return CASE_SETTINGS[name]
    for k, v in sorted(CASE_SETTINGS.items(), key=lambda kv: -len(kv[0])):
        if name == k or name.startswith(k + "_"):
            return v
    return {}


def make_case(name, device="cpu", precision="double", shape=None, comm=None, **kw):
    m = registry.get(name)
    shape = shape or (SMALL_2D if m.dims == 2 else SMALL_3D)
    lat = Lattice(name, shape, device=torch.device(device), precision=precision, comm=comm, **kw)
    nx = shape[0]
    fl = np.full((lat.NZ, lat.NY, nx), collision_value(m, name), dtype=np.uint32)
    wall = m.node_type("Wall")
    if wall is not None and not case_settings(name).get("_no_walls"):
        fl[:, :, 0] = wall.value   # x = 0 plane of walls (not on the decomposed axis)
    lat.set_flags(fl)
    for k, v in case_settings(name).items():
        if not k.startswith("_") and m.setting(k) is not None:      # option-dependent settings (e.g. viscstep)
            lat.set_setting(k, v)
    return lat


def perturb(lat, amp=0.01):
    f = lat.fields_interior().clone()
    ox, oy, oz = lat.slab.offset
    nx, ny, nz = lat.shape
    Z, Y, X = np.meshgrid(np.arange(oz, oz + nz), np.arange(oy, oy + ny), np.arange(nx), indexing="ij")
    # a different phase per field: perturbing every population by the same factor makes
    # e.g. the phase-field normal of d2q9_pf an O(grad^3) cancellation (rounding noise)
    ph = 0.3 * np.arange(f.shape[0])[:, None, None, None]
    p = 1 + amp * np.sin(0.37 * X[None] + 0.71 * Y[None] + 1.13 * Z[None] + ph)
    p = torch.from_numpy(p).to(f.device, f.dtype)
    lat.set_fields_interior(f * p)


def run(name, device="cpu", steps=3, precision="double", comm=None, shape=None):
    lat = make_case(name, device, precision, shape=shape, comm=comm)
    lat.init()
    perturb(lat)
    lat.iterate(steps)
    return lat
