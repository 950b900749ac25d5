"""Times the reference's own JS path (lib/kmers.js readFile(), unmodified, via
tools/ref_loader.js) on BASELINE C2: 10 M synthetic 150 bp reads (the bench's
splitmix64 generator, seed 1, 3.17 GB), k=16, prefix ATGAC -- once with
progress=false and once with the default progress=true (its per-line stdout
writes go to /dev/null).  BUILD CONTAINER ONLY: the reference never travels to
the GPU box, so this is "build container, 1 core (node is
single-threaded), not the GPU box".  The reference's ordered digest is checked
against the oracle's on the same bytes.  Writes profiles/ref_js_c2.json, which
bench.py carries as cpu_baseline.reference_js."""
import hashlib
import json
import os
import platform
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from oracle import oracle
    reads = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "c2_ref_%d.fastq" % reads)
    data = oracle.synth_fastq(1, 0, reads)
    with open(path, "wb") as f:
        f.write(data)
    t0 = time.perf_counter()
    want = oracle.count_buffer(data, b"ATGAC", 16, 1)
    t_oracle = time.perf_counter() - t0
    js = json.dumps([[k.decode("latin-1"), v] for k, v in want], separators=(",", ":"))
    want_digest = hashlib.sha256(js.encode("utf-8")).hexdigest()[:16]
    del data
    runs = []
    for prog in ("0", "1"):
        p = subprocess.run(["node", "--max-old-space-size=16384", os.path.join(REPO, "tools", "ref_loader.js"),
                            "--time", path, "ATGAC", "16", prog], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                           text=True, timeout=7200)
        r = json.loads(p.stderr.strip().splitlines()[-1])
        r["digest_equals_oracle"] = r["digest"] == want_digest
        r["windows"] = reads * 270
        r["kmers_per_s"] = reads * 270 / r["seconds"]
        runs.append(r)
        print(json.dumps(r), flush=True)
    os.unlink(path)
    cpu = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(x.split(":", 1)[1].strip() for x in f if x.startswith("model name"))
    except Exception:
        pass
    out = {"what": "reference lib/kmers.js readFile() (unmodified, tools/ref_loader.js) on BASELINE C2",
           "where": "build container, 1 core (node is single-threaded), not the GPU box",
           "host": {"cpu": cpu, "vcpus": os.cpu_count(), "node": subprocess.run(["node", "--version"],
                    capture_output=True, text=True).stdout.strip(), "python": platform.python_version()},
           "workload": "C2: %d synthetic 150bp reads (splitmix64, seed 1, 317 B records), k=16, prefix ATGAC" % reads,
           "oracle_digest": want_digest, "oracle_seconds_1_thread": t_oracle,
           "runs": runs}
    with open(os.path.join(REPO, "profiles", "ref_js_c2.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
