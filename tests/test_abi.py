"""CPU-side checks of the drop-in boundary: the C-ABI library loads and
exports every symbol include/kmer_api.h declares (no compute without a GPU)."""
import ctypes
import os
import re

from tests.conftest import REPO


def header_symbols():
    text = ""
    for h in ("kmer_api.h", "kmer_match.h"):
        with open(os.path.join(REPO, "include", h)) as f:
            text += f.read()
    return sorted(set(re.findall(r"\b(kmer_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    lib = ctypes.CDLL(os.path.join(REPO, "kmerjs_amd", "libkmerhip.so"))
    syms = header_symbols()
    assert len(syms) >= 18
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_lists_header_symbols():
    from kmerjs_amd import _native
    assert sorted(_native.EXPORTS) == header_symbols()


def test_version_and_status_strings():
    from kmerjs_amd import _native
    assert "gfx950" in _native.version()
    assert _native.LIB.kmer_status_string(5) == b"too many keys"


def test_open_rejects_bad_params_without_gpu():
    from kmerjs_amd import _native
    for kw in ({"k": 0}, {"step": 0}):
        try:
            _native.Counter(**kw)
        except _native.KmerError as e:
            assert e.status == 2
        else:
            raise AssertionError("accepted %r" % kw)


def test_product_does_not_reference_oracle():
    # the product package must never route through the CPU restatement
    pkg = os.path.join(REPO, "kmerjs_amd")
    for root, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".js", ".cc", ".hip", ".hpp")):
                with open(os.path.join(root, fn), encoding="utf-8") as f:
                    src = f.read()
                assert "oracle" not in src.replace("oracle/kmer_oracle.c", ""), fn


EXPERIMENT_ENV = ("KMERHIP_TAB_ABLATE", "KMERHIP_TAB_RANGE", "KMERHIP_TAB_FINAL", "KMERHIP_NL", "KMERHIP_TAB_S1",
                  "KMERHIP_TAB_S2", "KMERHIP_ONE_STREAM", "KMERHIP_TAB_PROF", "KMERHIP_DENSE")


def test_shipping_library_has_no_experiment_switches():
    """the A/B switches exist only in a -DKMERHIP_EXPERIMENTS
    build (tools/); the default library cannot read them, so a stray variable
    in a user's environment changes nothing."""
    with open(os.path.join(REPO, "kmerjs_amd", "libkmerhip.so"), "rb") as f:
        blob = f.read()
    present = [n for n in EXPERIMENT_ENV if n.encode() in blob]
    assert not present, present


def test_header_has_no_result_corrupting_flag():
    with open(os.path.join(REPO, "include", "kmer_api.h")) as f:
        text = f.read()
    assert "ABLATE" not in text and "WRONG" not in text


def test_open_rejects_reserved_flag_bits_without_gpu():
    from kmerjs_amd import _native
    for bit in range(8, 16):
        try:
            _native.Counter(flags=1 << bit)
        except _native.KmerError as e:
            assert e.status == 2
        else:
            raise AssertionError("accepted flag bit %d" % bit)


def _h2d_copies():
    """Every hipMemcpyAsync(..., hipMemcpyHostToDevice, ...) in the library's
    sources: (file, line, source argument)."""
    out = []
    csrc = os.path.join(REPO, "kmerjs_amd", "csrc")
    for fn in sorted(os.listdir(csrc)):
        if not fn.endswith((".hip", ".hpp")):
            continue
        with open(os.path.join(csrc, fn), encoding="utf-8") as f:
            src = f.read()
        for m in re.finditer(r"hipMemcpyAsync\s*\(([^;]*?)hipMemcpyHostToDevice", src):
            args = [a.strip() for a in m.group(1).split(",")]
            out.append((fn, src.count("\n", 0, m.start()) + 1, args[1]))
    return out


def test_no_async_upload_reads_a_host_temporary():
    # A pageable hipMemcpyAsync may read its host buffer after the call has
    # returned (round 4: a std::vector died first and stray keys were written).
    # Host temporaries go through the pinned upload arena (upload(),
    # kmer_feed.hip); the copies left read the arena, the caller's buffers or
    # long-lived members (ctx->..., db->..., m->...).
    copies = _h2d_copies()
    assert copies, "pattern found no upload at all"
    bad = [(fn, ln, a) for fn, ln, a in copies
           if ".data()" in a or (a.startswith("&") and "->" not in a) or a in ("off", "cur", "hp", "units", "segs")]
    assert not bad, bad
    srcs = sorted(set(a for _, _, a in copies))
    assert srcs == sorted(set(["h", "bytes + pos", "keys", "ts", "&db->entries", "&m->hits0", "offsets", "counts"])), srcs
