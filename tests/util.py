"""Test helpers shared by CPU and GPU tests (not the oracle)."""
import hashlib
import json


def js_stringify(entries):
    """JSON.stringify([...map]) for (key_bytes, count) pairs of ASCII keys."""
    return json.dumps([[k.decode("latin-1"), int(v)] for k, v in entries], separators=(",", ":"),
                      ensure_ascii=False)


def digest(entries):
    return hashlib.sha256(js_stringify(entries).encode("utf-8")).hexdigest()


def first_diff(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i, x, y
    if len(a) != len(b):
        i = min(len(a), len(b))
        return i, a[i] if i < len(a) else None, b[i] if i < len(b) else None
    return None
