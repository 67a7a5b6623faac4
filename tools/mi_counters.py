"""Summarise the SQ counter passes of tools/mi_pmc.sh (gpurun_out/mipmc/p1, p2) for
the batch MI kernel into profiles/<name>.txt / .json (read by bench.py's
mi_roofline for the VALU-issue fraction).

SQ_WAVE_CYCLES, SQ_BUSY_CYCLES-relative waits and SQ_ACTIVE_* count quad-cycles
per wave; SQ_BUSY_CYCLES counts cycles per shader engine (32 on MI355X).
Usage: tools/mi_counters.py NAME [PAIRS] [DIR]"""
import collections
import csv
import json
import os
import re
import sys

name = sys.argv[1]
pairs = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
d = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/mipmc"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
agg, cnt, kname = collections.defaultdict(float), collections.Counter(), None
for p in ("p1", "p2"):
    for r in csv.DictReader(open(os.path.join(d, p, "run_counter_collection.csv"))):
        k = r["Kernel_Name"]
        if "mi_quad_kernel" not in k and "mi_lane_kernel" not in k:
            continue
        kname = re.sub(r"^void |\(anonymous namespace\)::", "", k).split("(")[0].strip()
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[r["Counter_Name"]] += 1
c = {k: agg[k] / cnt[k] for k in agg}
SES, SIMDS, CLK = 32, 1024, 2.4e9
out = {
    "kernel": kname, "pairs": pairs, "counters": {k: c[k] for k in sorted(c)},
    "valu_insts_per_pair": c["SQ_INSTS_VALU"] / pairs,
    "lds_insts_per_pair": c["SQ_INSTS_LDS"] / pairs,
    "resident_waves_per_cu": 4 * c["SQ_WAVE_CYCLES"] / c["SQ_BUSY_CYCLES"] / 8,  # 8 CUs per shader engine
    "valu_active_per_wave": c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"],
    "wait_any_per_wave": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
    # wave64 VALU issue: one instruction per SIMD per 4 cycles at 2.4 GHz
    "valu_issue_floor_ms": c["SQ_INSTS_VALU"] * 4 / SIMDS / CLK * 1e3,
}
json.dump(out, open(os.path.join(root, "profiles", name + ".json"), "w"), indent=1)
with open(os.path.join(root, "profiles", name + ".txt"), "w") as f:
    f.write(f"# rocprofv3 --pmc, tools/mi_pmc.sh ({pairs} 11x11 pairs, tools/mi_bench.py; two passes)\n")
    f.write(f"# kernel {kname}\n")
    for k in sorted(c):
        f.write(f"{k}={c[k]:.4g}\n")
    for k in ("valu_insts_per_pair", "lds_insts_per_pair", "resident_waves_per_cu", "valu_active_per_wave",
              "wait_any_per_wave", "valu_issue_floor_ms"):
        f.write(f"{k}={out[k]:.4g}\n")
print(open(os.path.join(root, "profiles", name + ".txt")).read())
