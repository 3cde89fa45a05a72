"""d3q27_kl — regularised Kuang-Luo (viscoplastic + shear-thinning) blood rheology on
D3Q27 with BGK/TRT collision; the apparent viscosity is found per node by a fixed-point
iteration nu_app(gamma_dot) <-> gamma_dot(nu_app).  Optional OutFlow adds zero-gradient
(Neumann) outlets.  Reference: models/nonnewtonian/d3q27_kl/{Dynamics.R, Dynamics.c.Rt}."""
from ..dsl import Model

# reference density order f0..f26 (models/nonnewtonian/d3q27_kl/Dynamics.R:2-28)
U27 = [(0, 0, 0), (1, 0, 0), (0, 1, 0), (-1, 0, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1), (1, 1, 0), (-1, 1, 0),
       (-1, -1, 0), (1, -1, 0), (1, 0, 1), (0, 1, 1), (-1, 0, 1), (0, -1, 1), (1, 0, -1), (0, 1, -1),
       (-1, 0, -1), (0, -1, -1), (1, 1, 1), (-1, 1, 1), (-1, -1, 1), (1, -1, 1), (1, 1, -1), (-1, 1, -1),
       (-1, -1, -1), (1, -1, -1)]

STATE = ["gamma_dot", "nu_app", "Omega", "Dxx", "Dxy", "Dyz", "Dyy", "Dzx", "Dzz", "Iter", "lambda_even",
         "lambda_odd"]
OUTFLOW_DIRS = [("XP", (-1, 0, 0)), ("XN", (1, 0, 0)), ("YP", (0, -1, 0)), ("YN", (0, 1, 0)),
                ("ZP", (0, 0, -1)), ("ZN", (0, 0, 1))]


def build(outflow: bool = False) -> Model:
    m = Model("d3q27_kl" + ("_OutFlow" if outflow else ""), dims=3, family="nonnewtonian",
              reference="models/nonnewtonian/d3q27_kl",
              description="D3Q27 BGK/TRT with regularised Kuang-Luo viscoplastic shear-thinning rheology")
    for i, (x, y, z) in enumerate(U27):
        m.add_density(f"f[{i}]", x, y, z, group="f")
    if outflow:
        for i, (x, y, z) in enumerate(U27):
            m.add_field(f"f[{i}]", dx=(-x - 1, -x + 1), dy=-y, dz=-z)
            m.add_field(f"f[{i}]", dx=-x, dy=(-y - 1, -y + 1), dz=-z)
            m.add_field(f"f[{i}]", dx=-x, dy=-y, dz=(-z - 1, -z + 1))
    for n in STATE:
        m.add_density(n, 0, 0, 0, group="state")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("Shear")
    m.add_quantity("Nu_app")
    m.add_quantity("Stress")
    m.add_quantity("YieldStatus")
    for i in ("xx", "xy", "yz", "yy", "zx", "zz"):
        m.add_quantity(f"D{i}")
    m.add_quantity("Pressure")
    m.add_quantity("Iterations")
    m.add_quantity("Lambda_even")
    m.add_quantity("Lambda_odd")
    S = m.add_setting
    S("VelocityX", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("VelocityY", default=0, comment="inlet/outlet/init velocity", zonal=True)
    for a in "XYZ":
        S(f"Gravitation{a}", default=0, comment="body/external acceleration", zonal=True)
    S("Pressure", default=0.3333, comment="Pressure for boundary condition", zonal=True)
    S("Density", default=1, comment="Density")
    S("Strain_Dim", default=3, comment="Number of dimensions for strain calculation")
    S("deltaP", comment="half range of pressure fluctuations", zonal=True)
    S("Period", comment="Period of pressure fluctuations", zonal=True)
    S("Pmax", comment="Heartbeat Pmax", zonal=True)
    S("eta1", comment="Plastic viscosity component")
    S("eta2", comment="Shear thinning component")
    S("sigmaY", comment="Yield stress")
    S("m", comment="Regularisation parameter")
    S("Lambda", comment="TRT Magic Number")
    S("MaxIter", default=100)
    S("sLim", default=5e-16)
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("TRT", "COLLISION")
    for n in ("Solid", "Wall", "PressureXP", "PressureXN", "PressureSinXN", "PressureCosXN", "PressureHBXN"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("ExtendedBdy", "ADDITIONALS")
    if outflow:
        for d, _ in OUTFLOW_DIRS:
            m.add_node_type(f"Neumann{d}", "BOUNDARY")
    m.add_global("VelocityMax", op="MAX")
    m.add_node_type("LogP", "ADDITIONALS")
    for g in ("Log_Ux", "Log_Uy", "Log_Uz", "Log_P", "Log_rho"):
        m.add_global(g)
    m.options = {"OutFlow": outflow}
    m.set_dynamics("nonnewtonian/d3q27_kl.inc")
    return m
