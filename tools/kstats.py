"""Per-kernel summary from a rocprofv3 --kernel-trace database (results.db) or *_kernel_stats.csv."""
import csv
import re
import sqlite3
import sys


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, calls, tot, avg, pct in c.execute("select name,total_calls,total_duration,average,percentage "
                                                     "from top_kernels"):
            yield name, int(calls), float(tot), float(avg), float(pct)
    else:
        for x in csv.DictReader(open(path)):
            yield x["Name"], int(x["Calls"]), float(x["TotalDurationNs"]) / 1e3, float(x["AverageNs"]) / 1e3, \
                float(x["Percentage"])


if __name__ == "__main__":
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    tot = 0.0
    for k, (name, calls, total, avg, pct) in enumerate(rows(sys.argv[1])):
        tot += total
        if k < n:
            nm = re.sub(r"\(anonymous namespace\)::", "", name).split("(")[0]
            print("%-40s %6d %10.1f us %8.2f us/call %5.1f%%" % (nm[:40], calls, total, avg, pct))
    print("total kernel time %.1f us" % tot)
