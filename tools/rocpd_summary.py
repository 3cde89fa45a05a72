#!/usr/bin/env python3
"""Per-kernel summary (calls, total ms, mean ms, VGPR/SGPR, scratch, LDS) from a rocprofv3
rocpd SQLite database (rocprofv3 --kernel-trace ... writes <out>_results.db by default).

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db > profiles/<name>.csv
"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    q = """select s.kernel_name, count(*), sum(d.end - d.start) / 1e6, avg(d.end - d.start) / 1e6,
                  s.arch_vgpr_count, s.accum_vgpr_count, s.sgpr_count, s.private_segment_size,
                  s.group_segment_size, d.workgroup_size_x, d.workgroup_size_y, d.grid_size_x, d.grid_size_y,
                  d.grid_size_z
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           group by s.kernel_name order by 3 desc"""
    print("kernel,calls,total_ms,mean_ms,vgpr,agpr,sgpr,scratch_B,lds_B,wg_x,wg_y,grid_x,grid_y,grid_z")
    for r in c.execute(q):
        name = r[0].replace(",", ";")
        print(f"{name},{r[1]},{r[2]:.4f},{r[3]:.4f}," + ",".join(str(v) for v in r[4:]))


if __name__ == "__main__":
    main(sys.argv[1])
