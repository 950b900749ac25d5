"""The Node.js drop-in (kmerjs_amd/node/kmers.js over the N-API addon)."""
import json
import os
import shutil
import subprocess

import pytest

from tests.conftest import REPO

NODE = shutil.which("node")
RUNNER = os.path.join(REPO, "tests", "node", "run_node_tests.js")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def _run(mode, timeout):
    p = subprocess.run([NODE, RUNNER, mode], capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr
    res = json.loads(p.stdout.strip().splitlines()[-1])
    bad = [r for r in res if not r["ok"]]
    assert res and not bad, bad[:5]
    return res


def test_node_dropin_cpu():
    _run("cpu", 60)


@pytest.mark.gpu
def test_node_dropin_gpu_parity(golden):
    res = _run("gpu", 600)
    assert len(res) > 20
