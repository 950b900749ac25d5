"""Oracle answers for the BASELINE workloads at their FULL sizes, written to
tests/golden/fullsize.json for tests/test_full_size_gpu.py.

Test infrastructure (the CPU restatement, oracle/kmer_oracle.c), run once in
the build container:

    python tests/golden/gen_fullsize.py [--procs 8]

* C2  (10 M reads, seed 1, k 16, ATGAC) and the C4 per-GPU shard (125 M reads,
  seed 4, the 1 B-read job's share of one of 8 GPUs): readFile()'s ordered Map
  (lib/kmers.js:106-185) by oracle_count_synth on `procs` record-aligned
  shards, merged on the host: counts added, first occurrence = the earliest
  (shard, ordinal) -- every occurrence in shard s precedes those in shard
  s + 1 -- then the Map digest of SURVEY.md App. C (sha256 of
  JSON.stringify([...map])).  C2's must equal the reference's own digest
  (profiles/ref_js_c2.json: lib/kmers.js run unmodified on the same bytes).
* C3  (100 M reads, seed 3, k 31, no prefix, table mode): the table digest
  (kmer_table_digest's definition: a sum over forward windows, no map) by
  oracle_table_digest_synth on `procs` threads.
* C5  (1 GB of contigs per GPU, seed 5 = rank 0's, k 21, canonical table mode):
  the table digest of bench.make_contigs' single-line file read by the
  reference's rule (lines with index % 4 == 1, lib/kmers.js:151;
  oracle_table_digest) -- "c5" -- and of the 60-column .fsa file counted by
  record (KMER_FLAG_FASTA; oracle_table_digest_fasta) -- "c5fa".
"""
import argparse
import hashlib
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def _shard(args):
    seed, r0, r1, prefix, k = args
    from oracle import oracle
    keys, cnt, first, lines = oracle.count_synth_arrays(seed, r0, r1 - r0, prefix, k)
    return keys, cnt, first, lines


def ordered_map(seed, n_reads, prefix, k, procs):
    cuts = [n_reads * i // procs for i in range(procs + 1)]
    with mp.Pool(procs) as pool:
        parts = pool.map(_shard, [(seed, cuts[i], cuts[i + 1], prefix, k) for i in range(procs)])
    keys = np.concatenate([p[0] for p in parts])
    cnt = np.concatenate([p[1] for p in parts])
    first = np.concatenate([(np.uint64(i) << np.uint64(48)) | p[2] for i, p in enumerate(parts)])
    lines = sum(p[3] for p in parts)
    rows = np.ascontiguousarray(keys).view(np.dtype((np.void, k))).reshape(-1)
    uniq, inv = np.unique(rows, return_inverse=True)
    tot = np.zeros(len(uniq), np.uint64)
    np.add.at(tot, inv, cnt)
    fst = np.full(len(uniq), np.iinfo(np.uint64).max, np.uint64)
    np.minimum.at(fst, inv, first)
    order = np.argsort(fst, kind="stable")
    ukeys = uniq.view(np.uint8).reshape(-1, k)[order]
    ucnt = tot[order]
    h = hashlib.sha256()
    h.update(b"[")
    for i in range(len(ucnt)):
        h.update(b'%s["%s",%d]' % (b"," if i else b"", ukeys[i].tobytes(), int(ucnt[i])))
    h.update(b"]")
    return {"size": int(len(ucnt)), "sum": int(ucnt.sum()), "lines": int(lines), "digest": h.hexdigest()[:16]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--only", default="c2,c4,c3,c5,c5fa")
    a = ap.parse_args()
    out_path = os.path.join(REPO, "tests", "golden", "fullsize.json")
    out = json.load(open(out_path)) if os.path.exists(out_path) else {}
    from oracle import oracle
    for cfg in a.only.split(","):
        t = time.time()
        if cfg == "c2":
            r = ordered_map(1, 10_000_000, b"ATGAC", 16, a.procs)
            r.update(workload="C2: 10 M reads, seed 1, k 16, prefix ATGAC (ordered Map)")
        elif cfg == "c4":
            r = ordered_map(4, 125_000_000, b"ATGAC", 16, a.procs)
            r.update(workload="C4 per-GPU shard: 125 M reads, seed 4, k 16, prefix ATGAC (ordered Map)")
        elif cfg == "c3":
            d, w = oracle.table_digest_synth(3, 0, 100_000_000, 31, a.procs)
            r = {"table_digest": d, "forward_windows": w,
                 "workload": "C3: 100 M reads, seed 3, k 31, no prefix (table digest)"}
        elif cfg in ("c5", "c5fa"):
            import bench
            data, _ = bench.make_contigs(5, 1_000_000_000, 21, width=60 if cfg == "c5fa" else 0)
            d, w = (oracle.table_digest_fasta if cfg == "c5fa" else oracle.table_digest)(data, 21)
            r = {"table_digest": d, "forward_windows": w, "bytes": len(data),
                 "workload": "C5%s: bench.make_contigs(seed 5, 1 GB%s), k 21, canonical table mode (table digest)"
                             % (" FASTA" if cfg == "c5fa" else "",
                                ", 60 columns, counted by record" if cfg == "c5fa" else
                                ", single-line, lines % 4 == 1 counted")}
        else:
            raise SystemExit("unknown config " + cfg)
        r["seconds"] = round(time.time() - t, 1)
        r["procs"] = a.procs
        out[cfg] = r
        print(cfg, r, flush=True)
        with open(out_path, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
