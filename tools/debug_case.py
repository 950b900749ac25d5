"""Run golden cases on the GPU and print the first differences (debug aid)."""
import json
import sys

sys.path.insert(0, ".")
from kmerjs_amd import _native  # noqa: E402
from oracle import oracle  # noqa: E402

name, prefix, k = sys.argv[1], sys.argv[2].encode(), int(sys.argv[3])
data = open("tests/golden/inputs/" + name, "rb").read()
want = oracle.count_buffer(data, prefix, k, 1)
ctr = _native.Counter(k=k, prefix=prefix)
res = ctr.count_buffer(data)
got = res.entries()
print("want", len(want), "got", len(got), "lines", res.lines)
wd, gd = dict(want), dict(got)
for kk in sorted(set(wd) | set(gd)):
    if wd.get(kk) != gd.get(kk):
        print("  key", kk, "want", wd.get(kk), "got", gd.get(kk))
print("order ok" if [x for x, _ in want] == [x for x, _ in got] else "order differs")
print(json.dumps([[a.decode(), b] for a, b in got[:30]]))
print(json.dumps([[a.decode(), b] for a, b in want[:30]]))
