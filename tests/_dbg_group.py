import sys
sys.path.insert(0, ".")
from kmerjs_amd import _native as native
from oracle import oracle
from tests.util import first_diff
data = open("tests/golden/inputs/test_short.fastq", "rb").read()
want = oracle.count_buffer(data, b"ATGAC", 16, 1)
one = native.Counter(k=16, prefix=b"ATGAC")
r1 = one.count_buffer(data)
print("single", r1.entries(), r1.firsts)
for devs, bb in (([0, 0], 0), ([0, 0], 1 << 30), ([0], 0), ([0, 0, 0], 0), ([0, 0], 800)):
    g = native.Counter(k=16, prefix=b"ATGAC", devices=devs, batch_bytes=bb)
    r = g.count_buffer(data)
    print(devs, bb, r.entries(), r.firsts, r.lines, "OK" if r.entries() == want else "BAD")
    g.close()
data = oracle.synth_fastq(13, 0, 3000)
want = oracle.count_buffer(data, b"ATGAC", 16, 1)
for bb in (1 << 16, 1 << 30):
    g = native.Counter(k=16, prefix=b"ATGAC", devices=[0, 0, 0], batch_bytes=bb)
    r = g.count_buffer(data)
    print("synth", bb, len(r), len(want), first_diff(r.entries(), want))
    g.close()
