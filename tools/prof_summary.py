"""Summarise a rocprofv3 results database (kernel trace) into a text table for profiles/."""
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
print(f"# rocprofv3 --kernel-trace --stats summary of {db}")
print("name | calls | total_ns | average_ns | percent")
for r in c.execute("select name,total_calls,total_duration,average,percentage from top_kernels"):
    print(" | ".join(str(x) for x in r))
print("\n# dispatch geometry (distinct kernels)")
print("name | grid_x | workgroup_x | lds_size | vgpr | agpr | sgpr | scratch | mean_duration_ns")
for r in c.execute("select name,grid_x,workgroup_x,lds_size,vgpr_count,accum_vgpr_count,sgpr_count,scratch_size,"
                   "avg(duration) from kernels group by name,grid_x order by avg(duration) desc"):
    print(" | ".join(str(x) for x in r))
