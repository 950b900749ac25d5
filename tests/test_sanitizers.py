"""Sanitizer builds of the host code, CPU only: the C
restatement under AddressSanitizer + UBSan over every golden input and
configuration (results must equal the regular build's), and the N-API addon
built with ASan + UBSan under the Node drop-in's CPU tests.  (GPU-side ASan
is not available on the pool; the HIP library's host code is covered on the
GPU box by tools/sanitize_abi.sh.)"""
import json
import os
import shutil
import subprocess

import pytest

from tests.conftest import GOLDEN_DIR, REPO


def _fnv(entries):
    h = 1469598103934665603
    for k, v in entries:
        for b in k + b"\x00" + int(v).to_bytes(8, "little"):
            h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.fixture(scope="module")
def san_driver():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "san"], check=True, timeout=300)
    return os.path.join(REPO, "oracle", "_san", "san_driver")


def test_oracle_under_asan_ubsan(san_driver, golden):
    from oracle import oracle
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    cfgs = [("ATGAC", 16, 1), ("", 16, 1), ("", 31, 1), ("AT", 21, 2), ("N", 5, 1), ("", 4, 3), ("ACGT", 70, 1)]
    for name in golden["inputs"]:
        path = os.path.join(GOLDEN_DIR, "inputs", name)
        data = open(path, "rb").read()
        for p, k, step in cfgs:
            out = subprocess.run([san_driver, path, p, str(k), str(step)], capture_output=True, text=True,
                                 timeout=120, env=env)
            assert out.returncode == 0, (name, p, k, step, out.stderr[-3000:])
            got = out.stdout.split()
            try:
                want, st = oracle.count_buffer(data, p.encode(), k, step, stats=True)
            except oracle.OracleError:
                assert got[0] == "error", (name, got)
                continue
            assert [int(x) for x in got] == [len(want), sum(v for _, v in want), st["lines"], _fnv(want)], \
                (name, p, k, step)


@pytest.mark.skipif(shutil.which("node") is None or not os.path.isdir("/usr/include/node"),
                    reason="node / node headers not installed")
def test_node_addon_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "kmerjs_amd", "node"), "san"], check=True, timeout=300)
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, LD_PRELOAD=asan, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1",
               KMERHIP_ADDON=os.path.join(REPO, "kmerjs_amd", "node", "_san", "kmerhip.node"))
    p = subprocess.run(["node", os.path.join(REPO, "tests", "node", "run_node_tests.js"), "cpu"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res and all(r["ok"] for r in res), [r for r in res if not r["ok"]][:3]
    assert any(r["name"] == "addon loads" for r in res)
