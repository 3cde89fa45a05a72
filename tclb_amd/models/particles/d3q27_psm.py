"""d3q27_PSM — partially saturated method (Noble & Torczynski) for resolved particles on
D3Q27: per-node solid fraction from the particle coverage (CalcF stage, particle=True),
BGK/TRT fluid collision blended with a solid operator — non-equilibrium bounce-back
(NEBB) or superposition (SUP) — Guo forcing with an oscillating body acceleration,
optional Kuang-Luo viscoplastic rheology (KL), multi-particle coverage (MS), and
single-kernel coupling.  Reference: models/particles/d3q27_PSM/{Dynamics.R,
Dynamics.c.Rt} (OPT="MS*KL*TRT*(NEBB+SUP+(NEBB+SEP):singlekernel)").

The reference relaxes in the raw-moment basis; all operators are linear in f, so they
are applied here in population space with the symmetric/antisymmetric split (even /
odd raw moments) for TRT — same algebra, no 27x27 transforms."""
from ..dsl import Model

U27 = [[0, 0, 0], [1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1],
       [1, 1, 0], [-1, 1, 0], [1, -1, 0], [-1, -1, 0], [1, 0, 1], [-1, 0, 1], [1, 0, -1], [-1, 0, -1],
       [0, 1, 1], [0, -1, 1], [0, 1, -1], [0, -1, -1], [1, 1, 1], [-1, 1, 1], [1, -1, 1], [-1, -1, 1],
       [1, 1, -1], [-1, 1, -1], [1, -1, -1], [-1, -1, -1]]


def build(ms=False, kl=False, trt=False, nebb=False, sup=False, singlekernel=False, sep=False) -> Model:
    """``sep`` (the ``SEP:singlekernel`` products) is declared only in the reference's
    conf.mk; neither Dynamics.R nor Dynamics.c.Rt reads Options$SEP, so those variants are
    the particle-free single-kernel model (Options$particles = NEBB | SUP is false)."""
    m = Model("d3q27_PSM", dims=3, family="particles", reference="models/particles/d3q27_PSM",
              description="D3Q27 partially saturated method for resolved particles")
    particles = nebb or sup
    for i, (x, y, z) in enumerate(U27):
        m.add_density(f"f[{i}]", x, y, z, group="f")
    for i in range(27):   # neighbour access for the extrapolation boundaries (Dynamics.R)
        m.add_field(f"f[{i}]", dx=(1, -1), dy=(1, -1), dz=(1, -1))
    load, save = ["f"], ["f"]
    if particles:
        for n in ("sol", "uPx", "uPy", "uPz"):
            m.add_density(n, 0, 0, 0, group="Force", parameter=True)
        m.add_quantity("Solid", unit="1")
        m.add_global("TotalSVF", comment="Total of solids throughout domain")
    if kl:
        m.add_density("gamma_dot", 0, 0, 0, group="Viscosity")
        m.add_density("nu_app", 0, 0, 0, group="Viscosity")
        for q in ("Shear", "Nu_app", "Stress", "YieldStatus"):
            m.add_quantity(q)
        m.add_setting("Strain_Dim", default=3, comment="Number of dimensions for strain calculation")
        m.add_setting("eta1", comment="Plastic viscosity component")
        m.add_setting("eta2", comment="Shear thinning component")
        m.add_setting("n", comment="Flow behaviour index")
        m.add_setting("sigmaY", comment="Yield stress")
        m.add_setting("m", comment="Regularisation parameter")
        m.add_setting("MaxIter", default=100)
        m.add_setting("sLim", default=5e-16)
        load.append("Viscosity")
        save.append("Viscosity")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("Rho", unit="kg/m3")
    S = m.add_setting
    S("omegaF", comment="one over F relaxation time and initial relaxation time for kl")
    S("nu", default=0.1, comment="kinetic viscosity in LBM unit", unit="m2/s", omegaF="1.0/(3*nu+0.5)")
    if trt:
        S("Lambda", comment="TRT Magic Number")
    for a in "XYZ":
        S(f"Velocity{a}", default="0.0", zonal=True, comment=f"wall/inlet/outlet velocity {a.lower()}-direction")
    S("Pressure", default="0Pa", comment="Inlet pressure", zonal=True, unit="1Pa")
    S("aX_mean", default=0.0, comment="mean of oscillating acceleration X", zonal=True, unit="m/s2")
    S("aX_amp", default=0.0, comment="amplitude of oscillating acceleration X", zonal=True, unit="m/s2")
    S("aX_freq", default=0.0, comment="frequency of oscillating acceleration", zonal=True, unit="1/s")
    S("AccelY", default=0.0, comment="body acceleration Y", zonal=True, unit="m/s2")
    S("AccelZ", default=0.0, comment="body acceleration Z", zonal=True, unit="m/s2")
    for n in ("RegionMeasureX", "RegionMeasureY", "RegionMeasureZ", "PressureMeasure"):
        m.add_node_type(n, "ADDITIONALS")
    for g, u in [("TotalFluidMomentumX", "kgm/s"), ("TotalFluidMomentumY", "kgm/s"), ("TotalFluidMomentumZ", "kgm/s"),
                 ("TotalFluidMass", "kg"), ("TotalFluidVolume", "m3"), ("FlowRateX", "m/s"), ("FlowRateY", "m/s"),
                 ("FlowRateZ", "m/s"), ("PressureGauge", "Pa")]:
        m.add_global(g, unit=u)
    for f in "NEWSFB":
        m.add_node_type(f"{f}Velocity", "BOUNDARY")
    for f in "NEWSFB":
        m.add_node_type(f"{f}Pressure", "BOUNDARY")
    for f in "NSEW":
        m.add_node_type(f"MovingWall_{f}", "BOUNDARY")
    if particles and singlekernel:
        m.add_stage("BaseInit", "Init", save_fields=save + ["Force"])
        m.add_stage("BaseIteration", "Run", save_fields=save + ["Force"], load_densities=load, particle=True)
        m.add_action("Iteration", ["BaseIteration"])
        m.add_action("Init", ["BaseInit"])
    elif particles:
        m.add_stage("BaseInit", "Init", save_fields=save)
        m.add_stage("BaseIteration", "Run", save_fields=save, load_densities=load + ["Force"])
        # lazy: the populations are pulled only within reach of a particle (d3q27_psm.inc CalcF)
        m.add_stage("CalcF", "CalcF", save_fields=["Force"], load_densities=load, particle=True, lazy_load=True)
        m.add_action("Iteration", ["BaseIteration", "CalcF"])
        m.add_action("Init", ["BaseInit", "CalcF"])
    else:
        m.add_stage("BaseInit", "Init", save_fields=save)
        m.add_stage("BaseIteration", "Run", save_fields=save, load_densities=load)
        m.add_action("Iteration", ["BaseIteration"])
        m.add_action("Init", ["BaseInit"])
    m.add_node_type("Solid", "BOUNDARY")
    m.add_node_type("Wall", "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    if singlekernel:
        m.glob_waves = 0          # a 2-wave cap spilled its globals kernel (r03s)
    m.options = {"SEP": sep, "MS": ms, "KL": kl, "TRT": trt, "NEBB": nebb, "SUP": sup, "singlekernel": singlekernel,
                 "particles": particles}
    m.set_dynamics("particles/d3q27_psm.inc")
    return m
