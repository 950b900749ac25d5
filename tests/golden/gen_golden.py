"""Generate golden vectors by running the UNMODIFIED reference (lib/kmers.js).

Build-container only: drives tools/ref_loader.js (which reads
/root/reference/lib/kmers.js at run time) over the fixture inputs in
tests/golden/inputs/ and writes tests/golden/golden.json.  Nothing here runs on
the GPU box; the committed golden.json is pure data (inputs' sha256 and the
reference's ordered [key, count] output or its digest).

Digest = sha256 of JSON.stringify([...map]) (the ordered Map).
"""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
INPUTS = os.path.join(HERE, "inputs")
FULL_LIMIT = 2500     # store full ordered entries up to this many keys

SMALL = ["test_short.fastq", "test_kmers.fastq", "edge_blank.fastq", "edge_crlf.fastq",
         "edge_notrail.fastq", "edge_exotic.fastq", "edge_pal.fastq", "edge_empty.fastq",
         "edge_newlines.fastq", "edge_len1.fastq"]
MEDIUM = ["test_long.kmer.fastq", "edge_longline.fastq", "edge_ragged.fastq", "edge_contigs.fsa",
          "syn_s1_r2000.fastq"]


def cases():
    out = []
    for f in SMALL:
        for p in ["ATGAC", "", "A", "GTCAT", "ATGACG", "N", "X", "AT"]:
            for k in [1, 2, 4, 5, 16, 21, 31, 32, 33, 40]:
                for step in [1, 2, 3]:
                    out.append((f, p, k, step))
    for f in MEDIUM:
        for p in ["ATGAC", "", "GT", "ATGACGC"]:
            for k in [16, 21, 31, 32, 33]:
                out.append((f, p, k, 1))
        out.append((f, "ATGAC", 16, 2))
        out.append((f, "ATGAC", 5, 1))
        out.append((f, "ATGAC", 7, 3))
    return out


def sha(b):
    return hashlib.sha256(b).hexdigest()


def main():
    cs = cases()
    batch = [{"id": i, "file": os.path.join(INPUTS, f), "prefix": p, "k": k, "step": s}
             for i, (f, p, k, s) in enumerate(cs)]
    proc = subprocess.run(["node", os.path.join(REPO, "tools", "ref_loader.js"), "--batch"],
                          input=json.dumps(batch).encode(), stdout=subprocess.PIPE, check=True)
    res = {}
    for line in proc.stdout.decode().splitlines():
        r = json.loads(line)
        res[r["id"]] = r
    assert len(res) == len(cs), (len(res), len(cs))
    in_sha = {}
    for f in set(c[0] for c in cs):
        with open(os.path.join(INPUTS, f), "rb") as fh:
            in_sha[f] = sha(fh.read())
    golden = {"inputs": in_sha, "cases": []}
    for i, (f, p, k, s) in enumerate(cs):
        r = res[i]
        ent_json = r["entries"]
        entries = json.loads(ent_json)
        c = {"input": f, "prefix": p, "k": k, "step": s, "lines": r["lines"],
             "size": len(entries), "sum": sum(v for _, v in entries),
             "digest": sha(ent_json.encode("utf-8"))}
        if len(entries) <= FULL_LIMIT:
            c["entries"] = entries
        else:
            c["head"] = entries[:64]
        golden["cases"].append(c)
    with open(os.path.join(HERE, "golden.json"), "w") as fh:
        json.dump(golden, fh, separators=(",", ":"))
    print("wrote %d cases" % len(cs), file=sys.stderr)


if __name__ == "__main__":
    main()
