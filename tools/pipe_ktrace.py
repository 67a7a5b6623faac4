"""Per-stream busy time and gaps of the VO loop's kernels from a rocprofv3
--kernel-trace database (tools/pipe_run.py): per keyframe (klt_kernel to
klt_kernel), each stream's kernel time, its idle time between kernels, and
the largest idle gaps by (previous kernel -> next kernel).
Usage: tools/pipe_ktrace.py TRACE_DIR"""
import collections
import glob
import re
import sqlite3
import sys

db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
con = sqlite3.connect(db)
cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
print("columns:", cols)
sc = "stream_id" if "stream_id" in cols else ("queue_id" if "queue_id" in cols else None)
rows = list(con.execute(f"select name,start,end,{sc or 0} from kernels order by start"))
nm = lambda s: re.sub(r"\(anonymous namespace\)::|void ", "", s).split("(")[0].split("<")[0]  # noqa: E731
idx = [i for i, r in enumerate(rows) if nm(r[0]) == "klt_kernel"]
if len(idx) < 14:
    sys.exit("too few keyframes in the trace")
t0, t1 = rows[idx[8]][1], rows[idx[-2]][1]
nf = len(idx) - 2 - 8
print(f"keyframes {nf}: {(t1 - t0) / 1e3 / nf:.1f} us per keyframe")
per = collections.defaultdict(list)
for r in rows:
    if t0 <= r[1] < t1:
        per[r[3]].append(r)
for s, rs in per.items():
    busy = sum(r[2] - r[1] for r in rs) / 1e3 / nf
    gaps = collections.Counter()
    idle = 0.0
    for a, b in zip(rs, rs[1:]):
        g = max(0, b[1] - a[2]) / 1e3
        idle += g
        gaps[(nm(a[0]), nm(b[0]))] += g / nf
    names = collections.Counter(nm(r[0]) for r in rs)
    print(f"stream {s}: {len(rs) / nf:.1f} kernels, busy {busy:.1f} us, idle {idle / nf:.1f} us per keyframe; "
          f"top kernels {names.most_common(6)}")
    for k, v in gaps.most_common(10):
        print("   idle %-70s %7.1f us" % ("%s -> %s" % k, v))
