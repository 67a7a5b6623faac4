# instruction-cache PMC pass over the config-3 BA families (cam_solve: is wave 0's chain fetch-bound?)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
CONFIGS=3 timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/icache" -o run -- python3 "$GRAFT_REPO_ROOT/tools/ab_ba_fams.py" > "$GRAFT_REPO_ROOT/gpurun_out/icache.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/icache.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
python3 - <<'PY'
import csv, collections, glob, re
f = glob.glob("gpurun_out/icache/**/run_counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = re.split(r"[(<]", re.sub(r"\(anonymous namespace\)::|^void ", "", r["Kernel_Name"]))[0]
    d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in d.items():
    print(k, {c: round(sum(x) / len(x), 1) for c, x in v.items()}, "launches", len(next(iter(v.values()))))
PY
