"""Per-kernel HBM traffic per launch from the two rocprofv3 --pmc passes of tools/pmc.sh.

traffic = 2 x FETCH_SIZE + WRITE_SIZE (bytes per launch, averaged over launches): on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced read, WRITE_SIZE is exact
(MI355X_MICROARCH.md, HBM section).  Writes profiles/<name>.json, read by bench.py."""
import collections
import csv
import json
import re
import sys


def name_of(k):
    k = re.sub(r"\(anonymous namespace\)::", "", k)
    k = re.sub(r"^void ", "", k)
    return re.split(r"[(<]", k)[0]


def per_kernel(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[name_of(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)  # KB -> B
    return d


if __name__ == "__main__":
    src, dst = sys.argv[1], sys.argv[2]
    f = per_kernel(f"{src}/FETCH_SIZE/run_counter_collection.csv")
    w = per_kernel(f"{src}/WRITE_SIZE/run_counter_collection.csv")
    out = {}
    for k in sorted(set(f) | set(w)):
        fa = sum(f.get(k, [0])) / max(len(f.get(k, [])), 1)
        wa = sum(w.get(k, [0])) / max(len(w.get(k, [])), 1)
        out[k] = {"launches": len(f.get(k, [])), "fetch_bytes_raw": round(fa), "write_bytes": round(wa),
                  "traffic_bytes": round(2 * fa + wa)}
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    for k, v in sorted(out.items(), key=lambda x: -x[1]["traffic_bytes"]):
        print("%-34s %5d  fetch(raw) %10d  write %10d  traffic %10d" % (k, v["launches"], v["fetch_bytes_raw"],
                                                                       v["write_bytes"], v["traffic_bytes"]))
