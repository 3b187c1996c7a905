"""Per-kernel duration summary from a rocprofv3 results database (sqlite), grouped by kernel
name and grid shape: python tools/dbstats.py gpurun_out/profX/run_results.db [name-filter]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else ""
q = ("select name, grid_x, grid_y, grid_z, count(*), avg(duration), min(duration) from kernels "
     "where name like ? group by name, grid_x, grid_y, grid_z order by min(id)")
for name, gx, gy, gz, n, avg, mn in c.execute(q, ("%" + flt + "%",)):
    short = name.split("(")[0][-48:]
    print("%-48s grid %7d x %4d x %2d  n=%4d  avg %8.2f us  min %8.2f us" % (short, gx, gy, gz, n, avg / 1e3, mn / 1e3))
