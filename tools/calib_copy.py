#!/usr/bin/env python3
"""Known-byte calibration for tools/counters.py: device copies of 1 GiB (fp64, 8 B/lane
and wider) so the FETCH_SIZE / WRITE_SIZE scale of the counters can be read against an
exact byte count, and a copy-bandwidth ceiling of this box (GB/s) is printed."""
import time

import torch


def main():
    n = 1 << 27  # 1 GiB of fp64
    a = torch.ones(n, dtype=torch.float64, device="cuda")
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    torch.cuda.synchronize()
    t = time.perf_counter()
    k = 20
    for _ in range(k):
        b.copy_(a)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / k
    print(f"copy 1 GiB fp64: {dt * 1e3:.3f} ms, {2 * 8 * n / dt / 1e9:.1f} GB/s (read+write)", flush=True)


if __name__ == "__main__":
    main()
