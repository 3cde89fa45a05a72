"""Worker of the multi-process GPU tests (tests/test_gpu_ipc.py): several processes on ONE
device, halos and particle forces through the native loop's IPC transport
(parallel/native.py, csrc/device/dist.hip xstart_ipc), control over gloo."""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))


def run_case(case, shape, steps, comm, grid=None):
    """the lattice of `case` on cuda:0, stepped `steps` times; d3q27: the channel of
    tests/dist_worker.py with its global-coordinate perturbation; part: the part256
    particle case (tools/bench_configs.py) at `shape`"""
    dev = torch.device("cuda", 0)
    if case == "part":
        import bench_configs as bc
        lat = bc.part256(shape, "double", dev, comm=comm)
        lat.iterate(steps)
        return lat
    import dist_worker
    if case == "part3":
        return dist_worker.particle_case(shape, steps, comm, device=dev)
    from tclb_amd.lattice import Lattice
    lat = Lattice("d3q27", shape, comm=comm, grid=grid, device=dev)
    lat.set_flags(dist_worker.setup_flags(lat))
    lat.set_setting("nu", 0.05)
    lat.set_setting("ForceX", 1e-4)
    lat.set_setting("Velocity", 0.01)
    lat.init()
    f = lat.fields_interior().clone()
    ox, oy, oz = lat.slab.offset
    nx, ny, nz = lat.shape
    Z, Y, X = np.meshgrid(np.arange(oz, oz + nz), np.arange(oy, oy + ny), np.arange(nx), indexing="ij")
    pert = torch.from_numpy(1 + 0.01 * np.sin(0.3 * X + 0.7 * Y + 1.1 * Z)).to(dev)
    lat.set_fields_interior(f * pert[None])
    lat.iterate(steps)
    return lat


def summary(lat):
    ps = lat.particles
    part = None
    if ps is not None:
        part = {"x": np.asarray(ps.x, dtype=float).tolist(), "v": np.asarray(ps.v, dtype=float).tolist(),
                "force": np.asarray(ps.force, dtype=float).tolist()}
    return part


def worker(rank, world, port, case, shape, steps, out, grid=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["TCLB_DIST_TRANSPORT"] = "ipc"
    os.environ.setdefault("TCLB_IPC_TIMEOUT_S", "30")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tclb_amd.parallel.comm import TorchDistComm
    comm = TorchDistComm()
    lat = run_case(case, shape, steps, comm, grid=grid)
    torch.cuda.synchronize()
    lat._dist.wait()                      # raises if a wait for a peer timed out
    parts = comm.gather_objects((lat.slab.offset, lat.fields_interior().cpu().numpy(), lat.globals,
                                 lat.slab.axis, lat._dist.transport, summary(lat)))
    if rank == 0:
        gnx, gny, gnz = lat.gshape
        full = np.zeros((lat.nf, gnz, gny, gnx))
        for (ox, oy, oz), a, *_ in parts:
            full[:, oz:oz + a.shape[1], oy:oy + a.shape[2], :] = a
        np.save(out, full)
        with open(out + ".json", "w") as f:
            json.dump({"globals": parts[0][2], "axis": parts[0][3], "transport": [p[4] for p in parts],
                       "part": parts[0][5]}, f)
    dist.barrier()
    dist.destroy_process_group()


def worker_dead_peer(rank, world, port, out):
    """rank 1 stops stepping after the first iterate; rank 0's next waits run into the
    bounded IPC timeout and NativeLoop.wait raises instead of hanging (no collective
    after that)"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["TCLB_DIST_TRANSPORT"] = "ipc"
    os.environ["TCLB_IPC_TIMEOUT_S"] = "3"
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tclb_amd.parallel.comm import TorchDistComm
    from tclb_amd.parallel.native import NativeDistError
    comm = TorchDistComm()
    lat = run_case("d3q27", (32, 16, 24), 1, comm)
    torch.cuda.synchronize()
    dist.barrier()
    import time
    if rank == 1:
        # a peer that stops stepping (stays alive, so the memory rank 0 has mapped stays
        # valid) until the survivor has reported
        t0 = time.time()
        while not os.path.exists(out) and time.time() - t0 < 120:
            time.sleep(0.2)
        os._exit(0)
    t0 = time.time()
    msg = "no error"
    try:
        lat.iterate(3, glob_last=False)
        lat._dist.wait()
    except NativeDistError as e:
        msg = str(e)
    with open(out + ".tmp", "w") as f:
        json.dump({"error": msg, "seconds": time.time() - t0}, f)
    os.replace(out + ".tmp", out)
    os._exit(0)                           # the group is out of step: no teardown
