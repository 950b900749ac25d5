"""Python mirror of the kmerjs `lib/kmers.js` surface, backed by libkmerhip.

Same names, argument meaning and defaults as the reference so tests read like
the reference's own (test/kmers.js):

    KmerJS(fastq='', preffix='ATGAC', length=16, step=1, coverage=1,
           progress=True, env='node')                    lib/kmers.js:67-82
    KmerJS.kmersInLine(line)                             lib/kmers.js:88-100
    KmerJS.readFile() -> ReadHandle(promise, event)      lib/kmers.js:106-185
    complement, complementMap, jsonToStrMap, stringToMap,
    objectToMap, mapToJSON                               lib/kmers.js:12-54

The Map is a Python dict (insertion-ordered, like a JS Map).  readFile()
counts on the GPU (kmer_count_file); kmersInLine stays a CPU loop over one
line, as in the reference (a per-line GPU call would be pure overhead).
Divergence on error paths only: a missing file rejects the promise (the
reference crashes with an unhandled stream error, lib/kmers.js:139).
"""
import json
import threading
from concurrent.futures import Future

from . import _native

# lib/kmers.js:12-17
complementMap = {"A": "T", "T": "A", "G": "C", "C": "G"}
_COMP = {ord(k): v for k, v in complementMap.items()}


def complement(string):
    """Reverse complement; only A/T/G/C are mapped (lib/kmers.js:31-38)."""
    return string.translate(_COMP)[::-1]


def _obj_to_str_map(obj):
    return {str(k): v for k, v in obj.items()}


def jsonToStrMap(jsonStr):        # lib/kmers.js:27-29 (takes an object, despite the name)
    return _obj_to_str_map(jsonStr)


def stringToMap(string):          # lib/kmers.js:40-42
    return _obj_to_str_map(json.loads(string))


def objectToMap(obj):             # lib/kmers.js:43-45
    return _obj_to_str_map(obj)


def mapToJSON(strMap):            # lib/kmers.js:46-54
    return dict(strMap)


class _Event:
    """Stand-in for the progress stream returned as `event` (lib/kmers.js:108-110)."""

    def __init__(self):
        self._handlers = {}

    def on(self, name, fn):
        self._handlers.setdefault(name, []).append(fn)
        return self

    def emit(self, name, *args):
        for fn in self._handlers.get(name, []):
            fn(*args)


class ReadHandle:
    def __init__(self, promise, event):
        self.promise = promise
        self.event = event

    def __getitem__(self, key):          # handle["promise"], like the JS object
        return getattr(self, key)


class KmerJS:
    def __init__(self, fastq="", preffix="ATGAC", length=16, step=1, coverage=1, progress=True, env="node",
                 device=0):
        self.fastq = fastq
        self.preffix = preffix
        self.kmerLength = length
        self.step = step
        self.progress = progress
        self.coverage = coverage
        self.evalue = 0.05
        self.kmerMap = {}
        self.kmerMapSize = 0
        self.env = env
        self.device = device
        self.lines = 0
        if env == "browser":
            self.fileDataRead = 0

    def kmersInLine(self, line):
        """lib/kmers.js:88-100 — counts into self.kmerMap."""
        k, step, p, m = self.kmerLength, self.step, self.preffix, self.kmerMap
        L = len(line)
        ini = 0
        for _ in range(0, L - k + 1):
            kmer = line[ini:ini + k]
            if kmer.startswith(p):
                m[kmer] = m.get(kmer, 0) + 1
            ini += step

    def readFile(self):
        """lib/kmers.js:106-185 — GPU count of the whole file."""
        fut = Future()
        ev = _Event()

        def run():
            try:
                c = _native.Counter(k=self.kmerLength, prefix=self.preffix.encode("latin-1"), step=self.step,
                                    device=self.device)
                try:
                    res = c.count_file(self.fastq)
                finally:
                    c.close()
                for key, cnt in res.entries():
                    s = key.decode("latin-1")
                    self.kmerMap[s] = self.kmerMap.get(s, 0) + int(cnt)
                self.lines = int(res.lines)
                self.kmerMapSize = len(self.kmerMap)
                ev.emit("progress", {"percentage": 100})
                fut.set_result(self.kmerMap)
            except Exception as e:  # reject
                fut.set_exception(e)

        threading.Thread(target=run, daemon=True).start()
        return ReadHandle(fut, ev)
