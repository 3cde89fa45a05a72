"""Worker for multi-process (gloo, CPU) tests of the decomposition + halo path."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def setup_flags(lat):
    m = lat.model
    nx = lat.shape[0]
    fl = np.full((lat.NZ, lat.NY, nx), m.node_type("MRT").value, dtype=np.uint32)
    if m.name == "d3q27":
        # walls at global y = 0 and y = gny-1 (rows of every local y incl. ghosts)
        gy = (np.arange(lat.NY) + lat.slab.offset[1] - lat.gy) % lat.gshape[1]
        fl[:, gy == 0, :] = m.node_type("Wall").value
        fl[:, gy == lat.gshape[1] - 1, :] = m.node_type("Wall").value
    return fl


def run_case(model, shape, steps, comm, overlap=None, grid=None):
    from tclb_amd.lattice import Lattice
    lat = Lattice(model, shape, comm=comm, overlap=overlap, grid=grid)
    lat.set_flags(setup_flags(lat))
    if model == "d3q27":
        lat.set_setting("nu", 0.05)
        lat.set_setting("ForceX", 1e-4)
        lat.set_setting("Velocity", 0.01)
    else:
        lat.set_setting("Viscosity", 0.05)
        lat.set_setting("VelocityX", 0.01)
        lat.set_setting("GravitationX", 1e-5)
    lat.init()
    # deterministic perturbation in global coordinates
    f = lat.fields_interior().clone()
    ox, oy, oz = lat.slab.offset
    nx, ny, nz = lat.shape
    Z, Y, X = np.meshgrid(np.arange(oz, oz + nz), np.arange(oy, oy + ny), np.arange(nx), indexing="ij")
    pert = 1 + 0.01 * np.sin(0.3 * X + 0.7 * Y + 1.1 * Z)
    lat.set_fields_interior(f * torch.from_numpy(pert)[None])
    lat.iterate(steps)
    return lat


def worker(rank, world, port, model, shape, steps, out, overlap, grid=None, native="1"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["TCLB_DIST_NATIVE"] = native
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tclb_amd.parallel.comm import TorchDistComm
    comm = TorchDistComm()
    lat = run_case(model, shape, steps, comm, overlap=overlap, grid=grid)
    parts = comm.gather_objects((lat.slab.offset, lat.fields_interior().numpy(), lat.globals, lat.slab.axis))
    if rank == 0:
        gnx, gny, gnz = lat.gshape
        full = np.zeros((lat.nf, gnz, gny, gnx))
        for (ox, oy, oz), a, _, _ in parts:
            full[:, oz:oz + a.shape[1], oy:oy + a.shape[2], :] = a
        np.save(out, full)
        with open(out + ".axis", "w") as f:
            f.write(str(parts[0][3]))
        import json
        with open(out + ".json", "w") as f:
            json.dump({**parts[0][2], "_native": lat._dist.transport if lat._dist is not None else None}, f)
    dist.barrier()
    dist.destroy_process_group()


def alternate_actions(lat, steps):
    """Iteration and TempToSteadyState alternately (two native plans with different
    staging sizes on a Y x Z grid; ADVICE r05: a shared, regrown staging buffer left the
    first plan pointing at freed memory)"""
    for _ in range(steps):
        lat.iterate(1, action="Iteration")
        lat.iterate(1, glob_last=False, action="TempToSteadyState")


def particle_case(shape, steps, comm, device=None):
    """the config-5 model (auto_d3q19_part, tools/bench_configs.py part256) with three
    density-2 spheres placed to cross z-slab boundaries: one straddling the middle cut, one
    wrapping the periodic z = 0 plane, one moving in z so it changes owner rank during the
    run.  Forces are summed over the ranks, positions advanced by SimplePart"""
    from tclb_amd.lattice import Lattice
    from tclb_amd.particles import SimplePart
    nx, ny, nz = shape
    lat = Lattice("auto_d3q19_part", shape, comm=comm, **({"device": device} if device is not None else {}))
    fl = np.full((lat.NZ, lat.NY, nx), lat.model.node_type("MRT").value, dtype=np.uint32)
    lat.set_flags(fl)
    lat.set_setting("Viscosity", 0.05)
    lat.set_setting("ForceX", 1e-5)
    ps = SimplePart()
    r = 3.0
    m = 2.0 * 4.0 / 3.0 * np.pi * r ** 3
    ps.add(x=(nx / 2, ny / 2, nz / 2 + 0.3), r=r, v=(0.02, 0, 0), m=m)
    ps.add(x=(nx / 4 + 0.4, ny / 4, 0.7), r=r, v=(0, 0.01, -0.02), m=m)
    ps.add(x=(3 * nx / 4, 3 * ny / 4, nz / 4 - 1.2), r=r, v=(0, 0, 0.4), m=m)
    ps.periodic[:] = True
    ps.period[:] = shape
    lat.particles = ps
    lat.init()
    lat.iterate(steps)
    return lat


def worker_particles(rank, world, port, shape, steps, out):
    """particle_case on `world` gloo ranks through the native loop, sends and receives
    paired by issue order (TCLB_DIST_ORDER_MATCH from the parent)"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["TCLB_DIST_NATIVE"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tclb_amd.parallel.comm import TorchDistComm
    comm = TorchDistComm()
    lat = particle_case(shape, steps, comm)
    ps = lat.particles
    parts = comm.gather_objects((lat.slab.offset, lat.fields_interior().numpy(), lat._native_path("Iteration"),
                                 lat._dist.transport if lat._dist is not None else None,
                                 np.asarray(ps.x, dtype=float), np.asarray(ps.v, dtype=float),
                                 np.asarray(ps.force, dtype=float)))
    if rank == 0:
        gnx, gny, gnz = lat.gshape
        full = np.zeros((lat.nf, gnz, gny, gnx))
        for (ox, oy, oz), a, *_ in parts:
            full[:, oz:oz + a.shape[1], oy:oy + a.shape[2], :] = a
        np.save(out, full)
        np.savez(out + ".part.npz", x=np.stack([p[4] for p in parts]), v=np.stack([p[5] for p in parts]),
                 force=np.stack([p[6] for p in parts]))
        import json
        with open(out + ".json", "w") as f:
            json.dump({"path": [p[2] for p in parts], "transport": [p[3] for p in parts]}, f)
    dist.barrier()
    dist.destroy_process_group()


def worker_catalog(rank, world, port, model, steps, out, overlap, mirror="1", alternate=False):
    """any catalog model with the generic set-up of tests/model_cases.py (global-coordinate
    perturbation), gathered to rank 0 as in worker()"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["TCLB_HALO_MIRROR"] = mirror
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from model_cases import make_case, perturb
    from tclb_amd.parallel.comm import TorchDistComm
    comm = TorchDistComm()
    lat = make_case(model, "cpu", comm=comm)
    lat.overlap = lat.overlap and overlap
    lat.init()
    perturb(lat)
    if alternate:
        alternate_actions(lat, steps)
    else:
        lat.iterate(steps)
    parts = comm.gather_objects((lat.slab.offset, lat.fields_interior().numpy(), lat.globals))
    if rank == 0:
        gnx, gny, gnz = lat.gshape
        full = np.zeros((lat.nf, gnz, gny, gnx))
        for (ox, oy, oz), a, _ in parts:
            full[:, oz:oz + a.shape[1], oy:oy + a.shape[2], :] = a
        np.save(out, full)
        import json
        with open(out + ".json", "w") as f:
            json.dump(parts[0][2], f)
    dist.barrier()
    dist.destroy_process_group()


def worker_checkpoint(rank, world, port, model, path, steps_before, steps_after, out):
    """checkpoint round trip over a rank-count change: with steps_before > 0 run that many
    steps and write `path`; then (steps_before == 0) load `path` and run steps_after,
    gathering the fields to rank 0 (`out`)"""
    import types
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from model_cases import make_case, perturb
    from tclb_amd.io.checkpoint import load_state, save_state
    from tclb_amd.parallel.comm import TorchDistComm
    comm = TorchDistComm()
    lat = make_case(model, "cpu", comm=comm)
    lat.init()
    solver = types.SimpleNamespace(lattice=lat, rank=rank, comm=comm, iter=0)
    if steps_before > 0:
        perturb(lat)
        lat.iterate(steps_before)
        solver.iter = lat.iter
        save_state(solver, path)
    else:
        load_state(solver, path)
        lat.iterate(steps_after)
        parts = comm.gather_objects((lat.slab.offset, lat.fields_interior().numpy(), lat.iter))
        if rank == 0:
            gnx, gny, gnz = lat.gshape
            full = np.zeros((lat.nf, gnz, gny, gnx))
            for (ox, oy, oz), a, _ in parts:
                full[:, oz:oz + a.shape[1], oy:oy + a.shape[2], :] = a
            np.save(out, full)
            with open(out + ".iter", "w") as f:
                f.write(str(parts[0][2]))
    dist.barrier()
    dist.destroy_process_group()


def adjoint_case(model, comm=None, steps=10, grid=None, device="cpu"):
    """unsteady adjoint of a small case: d3q19_adj pressure-driven duct through a porous
    design block (z-slabs), d2q9_kuper two-stage stencil model (y-slabs) with a setting
    gradient; returns (lattice, adjoint)"""
    from tclb_amd.adjoint import Adjoint
    from tclb_amd.lattice import Lattice
    from tclb_amd.parallel.comm import LoopbackComm
    comm = comm or LoopbackComm()
    if model == "d3q19_adj":
        nx, ny, nz = 10, 6, 8
        lat = Lattice(model, (nx, ny, nz), comm=comm, grid=grid, device=torch.device(device))
        m = lat.model
        mrt = m.node_type("MRT").value
        fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
        fl[:, :, 0] = m.node_type("WPressure").value | mrt
        fl[:, :, nx - 1] = m.node_type("EPressure").value | mrt
        fl[:, :, 7] |= m.node_type("Outlet").value
        fl[:, :, 4:6] |= m.node_type("DesignSpace").value
        lat.set_flags(fl)
        for k, v in {"nu": 0.1, "InletDensity": 1.03, "FluxInObj": 1.0, "Theta": 1.0}.items():
            lat.set_setting(k, v)
        lat.init()
        wi = m.field_index("w")
        f = lat.fields_interior().clone()
        oz = lat.slab.offset[2]
        zz = torch.arange(lat.shape[2], dtype=f.dtype, device=f.device)[:, None, None] + oz
        f[wi, :, :, 4:6] = (0.6 + 0.03 * zz).expand(-1, lat.shape[1], 2)
        lat.set_fields_interior(f)
        ad = Adjoint(lat, settings=["Theta"])
    else:
        nx, ny = 16, 12
        lat = Lattice(model, (nx, ny, 1), comm=comm, device=torch.device(device))
        m = lat.model
        fl = np.full((lat.NZ, lat.NY, nx), m.node_type("MRT").value, dtype=np.uint32)
        gy = (np.arange(lat.NY) + lat.slab.offset[1] - lat.gy) % ny
        fl[:, gy == 0, :] = m.node_type("Wall").value
        fl[:, gy == ny - 1, :] = m.node_type("Wall").value
        lat.set_flags(fl)
        for k, v in {"nu": 0.1666, "Magic": 0.005, "FAcc": 1.0, "Temperature": 0.65, "GravitationX": 1e-5,
                     "Density": 1.0, "WallForceXInObj": 1.0}.items():
            lat.set_setting(k, v)
        lat.init()
        ad = Adjoint(lat, settings=["GravitationX"])
    ad.unsteady(steps)
    return lat, ad


def worker_adjoint(rank, world, port, model, out, grid=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tclb_amd.parallel.comm import TorchDistComm
    comm = TorchDistComm()
    lat, ad = adjoint_case(model, comm, grid=grid)
    nx, ny, nz = lat.shape
    a = ad.a0[:, lat.gz:lat.gz + nz, lat.gy:lat.gy + ny, :nx].numpy()
    name = "Theta" if model == "d3q19_adj" else "GravitationX"
    sg = ad.setting_gradient(name)
    parts = comm.gather_objects((lat.slab.offset, a))
    if rank == 0:
        gnx, gny, gnz = lat.gshape
        full = np.zeros((lat.nf, gnz, gny, gnx))
        for (ox, oy, oz), p in parts:
            full[:, oz:oz + p.shape[1], oy:oy + p.shape[2], :] = p
        np.save(out, full)
        import json
        with open(out + ".json", "w") as f:
            json.dump({"J": ad.J, "grad": sg}, f)
    dist.barrier()
    dist.destroy_process_group()
