"""Frame timeline from a rocprofv3 --kernel-trace database of bench.py (one frame = klt_kernel to klt_kernel)."""
import collections, glob, re, sqlite3, sys
db = glob.glob((sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/trace") + "/*.db")[0]
rows = list(sqlite3.connect(db).execute("select name,start,end from kernels order by start"))
nm = lambda r: re.sub(r"\(anonymous namespace\)::|void ", "", r[0]).split("(")[0].split("<")[0]  # noqa: E731
idx = [i for i, r in enumerate(rows) if nm(r) == "klt_kernel"]
frames = [(rows[b][1] - rows[a][1]) / 1e3 for a, b in zip(idx[4:-1], idx[5:])]
print("frames %d  median %.1f us  min %.1f" % (len(frames), sorted(frames)[len(frames) // 2], min(frames)))
i0, i1 = idx[10], idx[11]
busy = collections.defaultdict(float)
cnt = collections.Counter()
for r in rows[i0:i1]:
    busy[nm(r)] += (r[2] - r[1]) / 1e3
    cnt[nm(r)] += 1
tot = sum(busy.values())
print("frame %.1f us  kernel busy %.1f us  launches %d" % ((rows[i1][1] - rows[i0][1]) / 1e3, tot, i1 - i0))
for k, v in sorted(busy.items(), key=lambda x: -x[1])[:25]:
    print("  %-32s %4d  %8.1f us  %6.2f us/launch" % (k, cnt[k], v, v / cnt[k]))
gaps = collections.Counter()
for a, b in zip(rows[i0:i1], rows[i0 + 1:i1 + 1]):
    gaps[(nm(a), nm(b))] += (b[1] - a[2]) / 1e3
print("largest gaps:")
for k, v in gaps.most_common(8):
    print("  %-60s %.1f us" % ("%s -> %s" % k, v))
