"""Benchmark of the k-mer -> template matcher (SURVEY.md §8f row 3;
include/kmer_match.h) on one MI355X.

Workload: the query is the C2 count (10 M synthetic reads, k=16, prefix
ATGAC: 1.96 M distinct k-mers) left in HBM by the counter and joined without
a host copy (kmer_match_open_device).  The template DB has the shape of the
reference's test_data/summary.json (5,030 templates, 16.5 M k-mer entries):
synthetic templates of 3,285 distinct ATGAC 16-mers each; `--present` of them
take 60 % of their k-mers from the query (the genomes in the sample), the rest
are random (which, since the query covers ~47 % of the 4^11 suffix space,
still share ~47 % of their k-mers with it).
A step = findMatches('winner'): round 1 (join + per-template scores) and the
winner loop to the end (GPU argmax / removal, host statistics), max_hits 100.
Also timed: the DB build (once), and 'standard' scoring.
CPU baseline: the oracle's numpy restatement of round 1 on the same data
(one core); the winner loop has no vectorised CPU restatement (pure-Python
loops), so only round 1 is compared.
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def measure(d_keys, d_cnt, nq, k=16, reads=10_000_000, templates=5030, per=3285, present=8, steps=3,
            cpu_baseline=True):
    """Matcher benchmark on a count already in HBM (kmer_result_device of a
    C2 count): returns the JSON-able record (also used by bench.py)."""
    import torch
    from kmerjs_amd import kmerfinder as kf
    from tests.match_util import kmer_codes, BASES
    dev = torch.device("cuda", torch.cuda.current_device())
    # query codes on the host (for the DB's present templates and the CPU baseline)
    from kmerjs_amd.multi import _CudaArray
    kt = torch.as_tensor(_CudaArray(d_keys, nq * k, "|u1"), device=dev).cpu().numpy().reshape(nq, k)
    ct = torch.as_tensor(_CudaArray(d_cnt, nq, "<u8"), device=dev).cpu().numpy().view(np.uint64)
    lut = np.zeros(256, dtype=np.uint64)
    lut[np.frombuffer(b"ACGT", dtype=np.uint8)] = np.arange(4, dtype=np.uint64)
    qc = np.zeros(nq, dtype=np.uint64)
    for i in range(k):
        qc = (qc << np.uint64(2)) | lut[kt[:, i]]

    rng = np.random.default_rng(7)
    nt, per = templates, per
    codes = kmer_codes(rng, nt * per * 2, k)
    allc = np.empty(nt * per, dtype=np.uint64)
    for t in range(nt):
        c = np.unique(codes[t * per * 2:(t + 1) * per * 2])[:per]
        if t < present:
            take = int(per * 0.6)
            c = np.unique(np.concatenate([rng.choice(qc, size=take, replace=False), c]))[:per]
        allc[t * per:(t + 1) * per] = c
    starts = np.arange(nt + 1, dtype=np.uint64) * np.uint64(per)
    mat = np.empty((allc.size, k), dtype=np.uint8)
    for j in range(k):                         # (column by column: no n x k 64-bit temporaries)
        mat[:, j] = BASES[((allc >> np.uint64(2 * (k - 1 - j))) & np.uint64(3)).astype(np.uint8)]
    keys = mat.tobytes()
    del mat
    meta = [{"sequence": "NC_%06d" % t, "lengths": 2 * per, "ulength": per, "species": "synthetic"}
            for t in range(nt)]
    summary = {"templates": nt, "totalLen": 2 * per * nt, "uniqueLens": per * nt}

    t0 = time.perf_counter()
    db = kf.TemplateDB.from_arrays(k, keys, starts, meta, summary)
    db_ms = (time.perf_counter() - t0) * 1e3
    info = db.info()
    finder = kf.KmerFinder(db, "winner")

    def one_step():
        t0 = time.perf_counter()
        m = kf.Match(db, device_result=(d_keys, k, d_cnt, nq))
        t1 = time.perf_counter()
        res = finder.find_matches(None, query_size=nq, match=m)
        t2 = time.perf_counter()
        w = m.winner()
        m.close()
        return (t1 - t0) * 1e3, (t2 - t1) * 1e3, res, w

    one_step()            # warmup
    r1, loop, res = [], [], None
    for _ in range(steps):
        a, b, res, _ = one_step()
        r1.append(a)
        loop.append(b)
    m = kf.Match(db, device_result=(d_keys, k, d_cnt, nq))
    tl = m.templates()
    w0 = m.winner()
    m.close()
    hits = int(w0.hits)
    t0 = time.perf_counter()
    std = kf.KmerFinder(db, "standard").find_matches(None, query_size=nq,
                                                     match=kf.Match(db, device_result=(d_keys, k, d_cnt, nq)))
    std_ms = (time.perf_counter() - t0) * 1e3

    out = {"metric": "template matching (kmerFinder findMatches 'winner') per query", "unit": "ms",
           "value": float(np.median(r1) + np.median(loop)), "higher_is_better": False,
           "config": {"workload": "C2 result (%d reads, k=16, ATGAC) vs synthetic DB" % reads,
                      "query_kmers": int(nq), "templates": nt, "db_entries": info["entries"],
                      "db_distinct": info["distinct"], "present": present},
           "round1_ms": float(np.median(r1)), "winner_loop_ms": float(np.median(loop)),
           "winners": len(res), "winner_names": [dict(x)["template"] for x in res][:12],
           "hits_round1": hits, "templates_hit": len(tl), "db_build_ms": db_ms, "standard_ms": std_ms,
           "standard_significant": sum(x is not None for x in std),
           "round1_hits_per_s": hits / (np.median(r1) / 1e3), "query_kmers_per_s": nq / (np.median(r1) / 1e3),
           "data": "synthetic"}
    if cpu_baseline:
        from oracle import kmerfinder_oracle as ko
        tix = np.repeat(np.arange(nt, dtype=np.int64), per)
        t0 = time.perf_counter()
        u, t, first, h = ko.numpy_first_round(qc, ct, allc, tix)
        cpu_ms = (time.perf_counter() - t0) * 1e3
        order = np.lexsort((np.arange(nt), first))
        order = order[u[order] > 0]
        ok = h == hits and [x[0] for x in tl] == [int(i) for i in order] and \
            [(x[1], x[2]) for x in tl] == [(int(u[i]), int(t[i])) for i in order]
        out["cpu_baseline"] = {"value": cpu_ms, "unit": "ms (round 1 only)", "cores": 1, "kind": "port",
                               "sample": "the full workload, round 1 (numpy restatement, oracle/kmerfinder_oracle.py)"}
        out["round1_verified_vs_oracle"] = bool(ok)
    db.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10_000_000)
    ap.add_argument("--templates", type=int, default=5030)
    ap.add_argument("--per", type=int, default=3285)
    ap.add_argument("--present", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    from kmerjs_amd import _native, synth_fastq_device

    dev = torch.device("cuda", 0)
    k = 16
    buf = torch.empty(args.reads * 317, dtype=torch.uint8, device=dev)
    synth_fastq_device(buf.data_ptr(), 1, 0, args.reads)
    torch.cuda.synchronize()
    ctr = _native.Counter(k=k, prefix=b"ATGAC")
    ctr.reset()
    ctr.feed_device(buf.data_ptr(), buf.numel())
    ctr.finish(want_result=False)
    d_keys, d_cnt, _, nq = ctr.result_device()
    del buf
    out = measure(d_keys, d_cnt, nq, k, args.reads, args.templates, args.per, args.present, args.steps,
                  not args.no_cpu_baseline)
    ctr.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
