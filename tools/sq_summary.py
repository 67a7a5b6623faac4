"""Summary of tools/sq_pmc.sh's SQ counter passes for one kernel (averaged over
its launches): instructions per unit of work, resident waves, VALU / LDS /
VMEM activity and waits per wave, LDS bank conflicts relative to LDS-active
cycles -- the evidence for what bounds a kernel (latency, issue, LDS).
SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / SQ_ACTIVE_* / SQ_WAIT_* count quad-cycles
per wave (SQ_BUSY_CYCLES per shader engine, 32 on MI355X, 8 CUs each).
Usage: sq_summary.py TAG KERNEL_REGEX UNITS DIR  ->  profiles/TAG.txt, .json"""
import collections
import csv
import glob
import json
import os
import re
import sys

tag, rx, units, d = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
agg, cnt, kname = collections.defaultdict(float), collections.Counter(), None
for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not re.search(rx, k):
            continue
        kname = re.sub(r"^void |\(anonymous namespace\)::", "", k).split("(")[0].strip()
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[r["Counter_Name"]] += 1
if not cnt:
    sys.exit(f"no launches of /{rx}/ in {d}")
c = {k: agg[k] / cnt[k] for k in agg}
wc = c.get("SQ_WAVE_CYCLES", 0.0)
out = {"kernel": kname, "units_per_launch": units, "counters_per_launch": {k: round(c[k], 1) for k in sorted(c)}}
for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH",
          "SQ_INSTS_VALU_MFMA_F64"):
    if k in c:
        out[k.lower()[3:] + "_per_unit"] = round(c[k] / units, 2)
if wc:
    for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY",
              "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS"):
        if k in c:
            out[k.lower()[3:] + "_per_wave_cycle"] = round(c[k] / wc, 4)
if "SQ_BUSY_CYCLES" in c and wc:
    out["resident_waves_per_cu"] = round(4 * wc / c["SQ_BUSY_CYCLES"] / 8, 2)
if "SQ_LDS_BANK_CONFLICT" in c and "SQ_ACTIVE_INST_LDS" in c and c["SQ_ACTIVE_INST_LDS"]:
    out["lds_bank_conflict_per_lds_active"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_ACTIVE_INST_LDS"], 3)
os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
json.dump(out, open(os.path.join(root, "profiles", tag + ".json"), "w"), indent=1)
with open(os.path.join(root, "profiles", tag + ".txt"), "w") as fh:
    for k, v in out.items():
        if k != "counters_per_launch":
            fh.write(f"{k}: {v}\n")
    for k, v in out["counters_per_launch"].items():
        fh.write(f"  {k}: {v}\n")
print(open(os.path.join(root, "profiles", tag + ".txt")).read())
