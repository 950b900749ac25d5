import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN_DIR = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "slow: long-running full-size check")
    config.addinivalue_line("markers", "fullsize: BASELINE-size property test (runs after every parity test)")


def pytest_collection_modifyitems(config, items):
    # parity first: the full-size property tests run last, so that a stop (-x)
    # in one of them hides no parity row (stable sort keeps the file order)
    items.sort(key=lambda it: 1 if it.get_closest_marker("fullsize") else 0)


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN_DIR, "golden.json")) as f:
        g = json.load(f)
    # materialise the synthetic input the goldens were made from (not committed)
    syn = os.path.join(GOLDEN_DIR, "inputs", "syn_s1_r2000.fastq")
    if not os.path.exists(syn):
        from oracle import oracle
        with open(syn, "wb") as f:
            f.write(oracle.synth_fastq(1, 0, 2000))
    return g


@pytest.fixture(scope="session")
def inputs(golden):
    data = {}
    for name in golden["inputs"]:
        with open(os.path.join(GOLDEN_DIR, "inputs", name), "rb") as f:
            data[name] = f.read()
    return data
