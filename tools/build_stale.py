#!/usr/bin/env python3
"""Rebuild only the kernel libraries whose sources changed (hip, cpu and the adjoint
libraries of the ADJOINT models), in parallel: the incremental form of
__graft_entry__.build()."""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tclb_amd import build as B  # noqa: E402
from tclb_amd.models.dsl import ADJOINT_MODELS  # noqa: E402


def main():
    jobs = [(m, k) for m in B.registry.names() for k in ("hip", "cpu") if B.stale_reason(m, k)]
    jobs += [(m, k) for m in sorted(ADJOINT_MODELS | {"d2q9_kuper"}) for k in ("ad", "adhip") if B.stale_reason(m, k)]
    print(f"{len(jobs)} stale libraries", flush=True)
    with ThreadPoolExecutor(max_workers=int(os.environ.get("MAX_JOBS", "8"))) as ex:
        for (m, k), _ in zip(jobs, ex.map(lambda t: B.build_model(t[0], kinds=(t[1],), verbose=True), jobs)):
            pass
    B.build_host()
    B.build_device_runtime()


if __name__ == "__main__":
    main()
