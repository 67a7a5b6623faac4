"""Summaries of rocprofv3 output (tools/gpu.sh writes the raw output under
gpurun_out/; these write the committed summaries under profiles/).

  kstats FILE [N]              per-kernel table from a --kernel-trace --stats database (*.db) or
                               *_kernel_stats.csv: calls, total, average, share
  pmc SRC DST                  HBM traffic per launch from the FETCH_SIZE / WRITE_SIZE --pmc passes under SRC:
                               traffic = 2 x FETCH_SIZE + WRITE_SIZE (the MI355X guide's gfx950 correction,
                               calibrated for 16-B/lane streaming reads only: bench.py labels the absolute
                               figure uncalibrated for these kernels); writes DST (.json, read by bench.py)
  sq TAG KERNEL_RX UNITS DIR   SQ counter passes under DIR for one kernel: instructions per unit of work,
                               resident waves, VALU / LDS / VMEM activity and waits per wave cycle, LDS
                               bank conflicts per LDS-active cycle -> profiles/TAG.txt / .json (with
                               UNIT=pair also the valu_insts_per_pair / resident_waves_per_cu keys
                               bench.py's mi_roofline reads)
SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* count quad-cycles per
wave (SQ_BUSY_CYCLES per shader engine: 32 on MI355X, 8 CUs each)."""
import collections
import csv
import glob
import json
import os
import re
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(k):
    k = re.sub(r"\(anonymous namespace\)::", "", k)
    k = re.sub(r"^void ", "", k)
    return k


def kstats_rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, calls, tot, avg, pct in c.execute("select name,total_calls,total_duration,average,percentage "
                                                     "from top_kernels"):
            yield name, int(calls), float(tot), float(avg), float(pct)
    else:
        for x in csv.DictReader(open(path)):
            yield x["Name"], int(x["Calls"]), float(x["TotalDurationNs"]) / 1e3, float(x["AverageNs"]) / 1e3, \
                float(x["Percentage"])


def cmd_kstats(argv):
    n = int(argv[1]) if len(argv) > 1 else 30
    tot = 0.0
    for k, (name, calls, total, avg, pct) in enumerate(kstats_rows(argv[0])):
        tot += total
        if k < n:
            nm = short(name).split("(")[0]
            print("%-40s %6d %10.1f us %8.2f us/call %5.1f%%" % (nm[:40], calls, total, avg, pct))
    print("total kernel time %.1f us" % tot)


def cmd_pmc(argv):
    src, dst = argv[0], argv[1]

    def per_kernel(path):
        d = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            d[re.split(r"[(<]", short(r["Kernel_Name"]))[0]].append(float(r["Counter_Value"]) * 1024.0)  # KB -> B
        return d
    f = per_kernel(glob.glob(f"{src}/FETCH_SIZE/**/*counter_collection.csv", recursive=True)[0])
    w = per_kernel(glob.glob(f"{src}/WRITE_SIZE/**/*counter_collection.csv", recursive=True)[0])
    out = {}
    for k in sorted(set(f) | set(w)):
        fa = sum(f.get(k, [0])) / max(len(f.get(k, [])), 1)
        wa = sum(w.get(k, [0])) / max(len(w.get(k, [])), 1)
        out[k] = {"launches": len(f.get(k, [])), "fetch_bytes_raw": round(fa), "write_bytes": round(wa),
                  "traffic_bytes": round(2 * fa + wa)}
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    with open(os.path.splitext(dst)[0] + ".txt", "w") as fh:
        fh.write("# HBM traffic per launch: 2 x FETCH_SIZE + WRITE_SIZE (uncalibrated for non-16-B-streaming kernels)\n")
        for k, v in sorted(out.items(), key=lambda x: -x[1]["traffic_bytes"]):
            fh.write("%-34s %5d  fetch(raw) %10d  write %10d  traffic %10d\n" % (
                k, v["launches"], v["fetch_bytes_raw"], v["write_bytes"], v["traffic_bytes"]))
    print(open(os.path.splitext(dst)[0] + ".txt").read())


def cmd_sq(argv):
    tag, rx, units, d = argv[0], argv[1], float(argv[2]), argv[3]
    unit = argv[4] if len(argv) > 4 else "unit"
    agg, cnt, kname = collections.defaultdict(float), collections.Counter(), None
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if not re.search(rx, k):
                continue
            kname = short(k).split("(")[0].strip()
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[r["Counter_Name"]] += 1
    if not cnt:
        sys.exit(f"no launches of /{rx}/ in {d}")
    c = {k: agg[k] / cnt[k] for k in agg}
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    out = {"kernel": kname, "units_per_launch": units, "unit": unit,
           "counters_per_launch": {k: round(c[k], 1) for k in sorted(c)}}
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_INSTS_SMEM",
              "SQ_INSTS_BRANCH", "SQ_INSTS_VALU_MFMA_F64"):
        if k in c:
            out[k.lower()[3:] + f"_per_{unit}"] = round(c[k] / units, 2)
    if wc:
        for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_ANY",
                  "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in c:
                out[k.lower()[3:] + "_per_wave_cycle"] = round(c[k] / wc, 4)
    if "SQ_BUSY_CYCLES" in c and wc:
        out["resident_waves_per_cu"] = round(4 * wc / c["SQ_BUSY_CYCLES"] / 8, 2)
    if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_ACTIVE_INST_LDS"):
        out["lds_bank_conflict_per_lds_active"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_ACTIVE_INST_LDS"], 3)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "profiles", tag + ".json"), "w"), indent=1)
    with open(os.path.join(ROOT, "profiles", tag + ".txt"), "w") as fh:
        for k, v in out.items():
            if k != "counters_per_launch":
                fh.write(f"{k}: {v}\n")
        for k, v in out["counters_per_launch"].items():
            fh.write(f"  {k}: {v}\n")
    print(open(os.path.join(ROOT, "profiles", tag + ".txt")).read())


if __name__ == "__main__":
    if len(sys.argv) < 2 or sys.argv[1] not in ("kstats", "pmc", "sq"):
        sys.exit(__doc__)
    globals()["cmd_" + sys.argv[1]](sys.argv[2:])
