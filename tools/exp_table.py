"""Table-mode phase times on one synthetic C3-shaped input, with optional
final-kernel ablations (KMERHIP_TAB_ABLATE; experiments only, results wrong).
usage: python tools/exp_table.py READS [ablate ...]"""
import os
import subprocess
import sys

if len(sys.argv) > 2 and sys.argv[2] != "child":
    for ab in sys.argv[2:]:
        env = dict(os.environ, KMERHIP_TAB_ABLATE=ab)
        subprocess.run([sys.executable, __file__, sys.argv[1], "child"], env=env, check=True)
    sys.exit(0)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from kmerjs_amd import _native, synth_fastq_device  # noqa: E402

n = int(sys.argv[1])
buf = torch.empty(n * 317, dtype=torch.uint8, device="cuda")
synth_fastq_device(buf.data_ptr(), 3, 0, n)
torch.cuda.synchronize()
c = _native.Counter(k=31, prefix=b"", flags=_native.FLAG_UNORDERED)
for it in range(3):
    c.reset()
    c.feed_device(buf.data_ptr(), buf.numel())
    c.finish(want_result=False)
    ph = c.phase_times()
print("ablate=%s reads=%d %s stats=%s" % (os.environ.get("KMERHIP_TAB_ABLATE", "0"), n,
      " ".join("%s=%.2f" % kv for kv in ph.items()), c.table_stats()), flush=True)
c.close()
