"""kmerjs_amd — MI355X-native replacement for kmerjs's FASTQ k-mer loop.

Product path: libkmerhip.so (HIP kernels for gfx950 behind the C-ABI in
include/kmer_api.h).  Python (`kmerjs_amd.kmers`) and Node.js
(`kmerjs_amd/node/kmers.js`) front-ends mirror the reference's KmerJS API.
"""
from ._native import Counter, KmerError, Result, synth_fastq_device, version  # noqa: F401
from .kmers import (KmerJS, complement, complementMap, jsonToStrMap, mapToJSON, objectToMap,  # noqa: F401
                    stringToMap)

__all__ = ["Counter", "KmerError", "Result", "synth_fastq_device", "version", "KmerJS", "complement",
           "complementMap", "jsonToStrMap", "mapToJSON", "objectToMap", "stringToMap"]
