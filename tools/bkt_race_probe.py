"""Race probe for bucket_scatter_kernel (the ordered finish's bucket scatter).

Run once per library build (one HIP library per process):
    KMERHIP_LIB_EXPERIMENT=kmerjs_amd/libkmerhip_probe_nofix.so python tools/bkt_race_probe.py nofix
    KMERHIP_LIB_EXPERIMENT=kmerjs_amd/libkmerhip_probe_fix.so   python tools/bkt_race_probe.py fix
    python tools/bkt_race_probe.py shipping

The probe builds (`make -C kmerjs_amd/csrc probes`) delay waves 1..3 of every
scatter workgroup before they place their keys, so that wave 0 reaches the
rewrite of the LDS bucket starts first -- the interleaving that, without the
barrier, lost counts and keys intermittently.  Each case is compared with the
CPU oracle (test infrastructure); one JSON line per case.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from kmerjs_amd import _native  # noqa: E402
from oracle import oracle  # noqa: E402

CASES = [  # (k, prefix, reads): k = 3 / 8 one bucket; k = 16 'ATGAC' 256 buckets (C2's finish)
    (3, b"", 2000),
    (8, b"A", 20000),
    (16, b"ATGAC", 200000),
]


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "shipping"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    for k, p, nr in CASES:
        data = oracle.synth_fastq(7, 0, nr)
        want = dict(oracle.count_buffer(data, p, k, 1))
        ctr = _native.Counter(k=k, prefix=p)
        bad = 0
        worst = None
        for _ in range(reps):
            got = ctr.count_buffer(data).entries()
            g = dict(got)
            lost = sum(want.values()) - sum(g.values())
            missing = sum(1 for x in want if x not in g)
            wrong = sum(1 for x, v in want.items() if g.get(x) != v)
            if wrong or len(g) != len(want):
                bad += 1
                worst = {"lost_counts": lost, "missing_keys": missing, "wrong_keys": wrong,
                         "distinct": len(g), "want_distinct": len(want)}
        ctr.close()
        print(json.dumps({"build": tag, "k": k, "prefix": p.decode(), "reads": nr, "reps": reps,
                          "bad_reps": bad, "example": worst}), flush=True)


if __name__ == "__main__":
    main()
