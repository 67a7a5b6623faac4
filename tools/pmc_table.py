"""Print per-kernel averages of every counter in rocprofv3 --pmc csv outputs (dirs given)."""
import collections, csv, glob, re, sys
d = collections.defaultdict(lambda: collections.defaultdict(list))
for base in sys.argv[1:]:
    for f in glob.glob(base + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.split(r"[(<]", re.sub(r"^void |\(anonymous namespace\)::", "", r["Kernel_Name"]))[0]
            d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in d.items():
    if k.startswith("__amd"):
        continue
    print(k, " ".join("%s=%.4g" % (c, sum(v) / len(v)) for c, v in sorted(cs.items())))
