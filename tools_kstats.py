import csv, re, sys
r = list(csv.DictReader(open(sys.argv[1])))
for x in r[: int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    name = re.sub(r"\(anonymous namespace\)::", "", x["Name"]).split("(")[0]
    print("%-34s %6s %10.1f us %5.1f%%" % (name[:34], x["Calls"], float(x["AverageNs"]) / 1e3, float(x["Percentage"])))
