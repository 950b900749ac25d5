"""Print one step's kernel timeline from a rocprofv3 kernel trace CSV."""
import csv
import re
import sys

path = sys.argv[1]
which = int(sys.argv[2]) if len(sys.argv) > 2 else 5
anchor = sys.argv[3] if len(sys.argv) > 3 else 'scan_tile|scan_planes'   # (a kernel launched once per step)
r = list(csv.DictReader(open(path)))
r.sort(key=lambda x: int(x['Start_Timestamp']))
idx = [i for i, x in enumerate(r) if re.search(anchor, x['Kernel_Name'])]
a, b = idx[which], idx[which + 1]
t0 = int(r[a]['Start_Timestamp'])
prev = None
tot = {}
for x in r[a:b]:
    n = x['Kernel_Name']
    m = re.findall(r'detail::(\w+)', n)
    name = (m[1] if len(m) > 1 else m[0]) if m else re.sub(r'\(.*', '', n).replace('kmerhip::', '')
    s = int(x['Start_Timestamp'])
    e = int(x['End_Timestamp'])
    print("%8.1f %7.1f gap %6.1f  %s grid=%s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3 if prev else 0,
                                                 name[:60], x['Grid_Size_X']))
    tot[name] = tot.get(name, 0) + (e - s) / 1e3
    prev = e
print("step span %.1f us" % ((int(r[b]['Start_Timestamp']) - t0) / 1e3))
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print("%8.1f  %s" % (v, k))
