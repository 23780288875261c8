"""Kernel statistics of a rocprofv3 rocpd database (``--kernel-trace --stats`` without
``--output-format csv`` writes only ``<name>_results.db``).  Prints the same columns as rocprofv3's
``kernel_stats.csv`` (durations in ns, as that file has them) from the database's ``top_kernels`` view
(whose durations are in us).

    python tools/rocpd_stats.py gpurun_out/r04b/trace/t_results.db > profiles/r04/final/bench_kernel_stats.csv
"""
import csv
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for name, calls, total_us, avg_us, pct in con.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        w.writerow([name, calls, round(total_us * 1e3), round(avg_us * 1e3), f"{pct:.6f}"])


if __name__ == "__main__":
    main()
