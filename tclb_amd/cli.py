"""Command line: ``python -m tclb_amd <model> case.xml [XPATH edits...]``

Equivalent of the reference's per-model executable ``CLB/<model>/main case.xml``
(reference: src/main.cpp:173-425) with the CLI XPath editor
(src/xpath_modification.cpp:4-163).  Multi-GPU: launch with torchrun (one rank per
GPU); the halo exchange then goes over RCCL.
"""
from __future__ import annotations

import argparse
import os
import sys
import xml.etree.ElementTree as ET

from .ops.abi import PRECISIONS
from .utils.log import log


def main(argv=None):
    ap = argparse.ArgumentParser(prog="tclb_amd", description="MI355X-native lattice Boltzmann solver")
    ap.add_argument("model", help="model name (see --list)")
    ap.add_argument("config", nargs="?", help="XML case file")
    ap.add_argument("edits", nargs="*", help="XPath edits: 'XPATH = value', 'XPATH @attr = value', ...")
    ap.add_argument("--device", default=None, choices=[None, "cpu", "cuda"])
    ap.add_argument("--precision", default="double", choices=list(PRECISIONS))
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--describe", action="store_true")
    a = ap.parse_intermixed_args(argv)   # options may follow the model / case file
    from .models import registry
    if a.list or a.model == "list":
        print("\n".join(registry.names()))
        return 0
    if a.describe:
        print(registry.get(a.model).describe())
        return 0
    if a.config is None:
        ap.error("config file required")
    from . import handlers  # noqa: F401
    from .parallel.comm import init_distributed_from_env
    from .solver import Solver
    from .utils.xpath import apply_edits, load_case
    root = load_case(a.config)
    root, exit_now = apply_edits(root, a.edits)
    if exit_now:
        return 0
    comm = init_distributed_from_env(a.device or "auto")
    s = Solver(a.model, root, conffile=a.config, device=a.device, precision=a.precision, comm=comm)
    s.run()
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        # leave together: a rank that exits while its peers are still in a collective
        # makes their transport abort (gloo IoException)
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
