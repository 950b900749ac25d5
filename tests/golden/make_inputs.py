"""Build the small edge-case FASTQ inputs used as parity fixtures.

Run once in the build container (outputs are committed under
tests/golden/inputs/).  Every file is tiny and deterministic (seeded).  The
cases target the exact-semantics rules of SURVEY.md Appendix A that the
reference's own fixtures do not exercise: blank lines shifting the mod-4
framing (lib/kmers.js:151,160), CRLF ('\\r' kept in the line, :120), no
trailing newline (:131-133), non-ACGT bytes kept by complement (:31-38),
lowercase, palindromes, length-0/1/short lines, and lines longer than a device
tile so windows cross tile boundaries at many offsets.
"""
import os
import random


HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "inputs")


def splitmix_mix(z):
    m = (1 << 64) - 1
    z = (z + 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def synth_fastq(seed, first_read, n_reads):
    """Python twin of oracle_synth_fastq / the device generator (317 B/record)."""
    m = (1 << 64) - 1
    out = bytearray()
    for r in range(n_reads):
        i = first_read + r
        bases = []
        for w in range(5):
            x = splitmix_mix((seed * 0x9E3779B97F4A7C15 + i * 8 + w) & m)
            for b in range(32):
                if w * 32 + b < 150:
                    bases.append("ACGT"[(x >> (2 * b)) & 3])
        out += b"@r%010d\n" % i
        out += "".join(bases).encode() + b"\n+\n" + b"I" * 150 + b"\n"
    return bytes(out)


def rnd_seq(rng, n, alphabet="ACGT"):
    return "".join(rng.choice(alphabet) for _ in range(n))


def rec(h, s, q=None):
    return "@%s\n%s\n+\n%s\n" % (h, s, q if q is not None else "I" * len(s))


def main():
    os.makedirs(OUT, exist_ok=True)
    rng = random.Random(20261015)
    files = {}

    # blank lines shift the framing: the header after a blank becomes "sequence"
    s = rec("a", "ATGACGCAATACTCCTGGTCATTT") + "\n" + rec("b", "GGATGACCTGAGAGCCTTAAGTCATG")
    s += rec("c", rnd_seq(rng, 60)) + "\n\n" + rec("d", "ATGACATGACATGACATGACATGAC")
    files["edge_blank.fastq"] = s

    # CRLF line endings: '\r' stays inside every line
    recs = [rec("r%d" % i, rnd_seq(rng, 40) + "ATGAC" + rnd_seq(rng, 20)) for i in range(6)]
    files["edge_crlf.fastq"] = "".join(recs).replace("\n", "\r\n")

    # no trailing newline, file ends inside a sequence line
    files["edge_notrail.fastq"] = rec("x", "ATGACGTTTGTCATCC") + "@y\nATGACGTACGTACGTAGTCATGTCAT"

    # lowercase, N, X, mixed case, spaces, tabs, '@' in sequence lines
    seqs = ["atgacgcaatactcctgtcat", "ATGACnnnnGTCAT", "ATGACXXXXXXXXXXXXXXX", "ATgACGCAATACTCCTGGTCAT",
            "ATGAC GCAATACTCCT\tGTCAT", "@ATGACGCAATACTCCT+GTCAT", "NNNNNNNNNNNNNNNNNNNNNN",
            "ATGACGTCAT", "A", "AT", "ATGACGCAATACTCC", "ATGACGCAATACTCCT", "ATGACGCAATACTCCTA"]
    files["edge_exotic.fastq"] = "".join(rec("e%d" % i, q) for i, q in enumerate(seqs))

    # palindromes (x == rc x) and self-overlapping prefixes
    pals = ["ACGT" * 10, "GAATTC" * 8, "ATGACGTCAT" * 4, "GTCATATGAC" * 4, "AAAATTTT" * 6, "ATGCAT" * 7]
    files["edge_pal.fastq"] = "".join(rec("p%d" % i, q) for i, q in enumerate(pals))

    files["edge_empty.fastq"] = ""
    files["edge_newlines.fastq"] = "\n" * 9
    files["edge_len1.fastq"] = "@a\nA\n+\nI\n@b\nAT\n+\nII\n@c\n\n+\n\n"

    # long lines crossing several 16 KiB device tiles; prefix-rich so windows
    # straddle tile seams at many offsets
    long1 = "".join(rng.choice(["ATGAC", "GTCAT", "A", "C", "G", "T", "N"]) for _ in range(14000))
    long2 = rnd_seq(rng, 40000)
    files["edge_longline.fastq"] = rec("L1", long1) + rec("L2", long2) + rec("L3", rnd_seq(rng, 150))

    # ragged reads: random lengths 0..400, sprinkled N/n, occasional blank line,
    # prefix-enriched so every window class occurs
    parts = []
    for i in range(400):
        n = rng.choice([0, 1, 2, 5, 15, 16, 17, 30, 31, 32, 33, 100, 150, 151, 250, 400])
        sq = list(rnd_seq(rng, n))
        for j in range(0, max(0, n - 5), 37):
            if rng.random() < 0.5:
                sq[j:j + 5] = rng.choice(["ATGAC", "GTCAT"])
        for j in range(n):
            if rng.random() < 0.01:
                sq[j] = rng.choice("NnX")
        parts.append(rec("g%d" % i, "".join(sq)[:n]))
        if rng.random() < 0.02:
            parts.append("\n")
    files["edge_ragged.fastq"] = "".join(parts)

    # FASTA-style contigs (C5 semantics: only lines with index % 4 == 1 count)
    fa = []
    for i in range(12):
        fa.append(">c%08d\n%s\n" % (i, rnd_seq(rng, rng.choice([500, 2000, 9000]))))
    files["edge_contigs.fsa"] = "".join(fa)

    for name, text in files.items():
        with open(os.path.join(OUT, name), "wb") as f:
            f.write(text.encode("ascii"))

    # deterministic synthetic set (same generator as the device / oracle)
    with open(os.path.join(OUT, "syn_s1_r2000.fastq"), "wb") as f:
        f.write(synth_fastq(1, 0, 2000))


if __name__ == "__main__":
    main()
