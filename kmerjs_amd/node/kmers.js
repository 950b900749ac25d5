/* kmers.js — drop-in replacement for kmerjs's lib/kmers.js, backed by the
 * MI355X HIP counter (libkmerhip via the kmerhip.node N-API addon).
 *
 * Same exports, constructor, fields and readFile() contract as the reference,
 * so KmerFinderClient / KmerFinderServer (which `extends KmerJS`) work
 * unchanged:
 *   complementMap, jsonToStrMap, complement, stringToMap, objectToMap,
 *   mapToJSON, KmerJS                                   lib/kmers.js:12-186
 * plus the legacy npm-main loop `kmers(line, kmerMap, length, preffix, step)`
 * (lib/index.js:60-73).
 *
 * readFile() resolves to this.kmerMap: a mutable JS Map (a KmerMap, which
 * extends Map and is filled lazily from the packed native result, when the
 * Map was empty) whose iteration order is the reference's first-occurrence
 * order (consumers rely on it: lib/kmerFinderServer.js:175,742).  More than
 * this.maxKeys (2^24, the reference Map's limit) distinct keys reject the
 * promise with a RangeError, as Map.set throws in the reference.  kmersInLine() stays a synchronous CPU
 * loop over one line, as in the reference (lib/kmers.js:88-100).
 *
 * this.kmerMap is created by the constructor (an empty KmerMap) and readFile()
 * fills that same object, as the reference resolves the constructor's Map
 * (lib/kmers.js:76, :178).  `event` is a Readable stream, as the reference's
 * progress-stream is (lib/kmers.js:108, :183): 'progress' events, a
 * progress() method returning the last one, and the stream ends after the
 * count (no bytes flow through it: the file is read natively).
 *
 * Documented divergences (error/diagnostic paths only): a missing file
 * rejects the promise (the reference throws from an unhandled stream error,
 * lib/kmers.js:139); progress is printed once per file instead of once per
 * line (lib/kmers.js:166-169); env 'browser' is not served by the GPU addon.
 */
'use strict';
const fs = require('fs');
const stream = require('stream');
const path = require('path');
const { KmerMap } = require('./kmer_map.js');

// the reference Map's capacity: Map.set throws RangeError beyond 2^24 keys
// (lib/kmers.js:95); the native count is told the same limit and rejects
const MAP_MAX_KEYS = 16777216;
const KMER_E_TOO_MANY_KEYS = 5;

let addon = null;
function native() {
    if (!addon) {
        // fails loudly if the HIP library / addon is not built: no CPU fallback
        // (KMERHIP_ADDON: another build of the same addon, e.g. the sanitizer
        // build of tests/test_sanitizers.py)
        addon = require(process.env.KMERHIP_ADDON || path.join(__dirname, 'kmerhip.node'));
    }
    return addon;
}

let BN;
try {
    BN = require('bignumber.js');   // the reference's evalue type (lib/kmers.js:75)
} catch (e) {
    BN = class SmallBN {            // minimal stand-in with the comparison API consumers use
        constructor(v) { this.v = Number(v); }
        cmp(o) { const x = o instanceof SmallBN ? o.v : Number(o); return this.v < x ? -1 : this.v > x ? 1 : 0; }
        lt(o) { return this.cmp(o) < 0; }
        gt(o) { return this.cmp(o) > 0; }
        toNumber() { return this.v; }
        valueOf() { return this.v; }
        toString() { return String(this.v); }
    };
}

const complementMap = new Map([['A', 'T'], ['T', 'A'], ['G', 'C'], ['C', 'G']]);

function objToStrMap(obj) {
    const m = new Map();
    for (const k of Object.keys(obj)) m.set(k, obj[k]);
    return m;
}
function jsonToStrMap(jsonStr) { return objToStrMap(jsonStr); }
function stringToMap(string) { return objToStrMap(JSON.parse(string)); }
function objectToMap(object) { return objToStrMap(object); }
function mapToJSON(strMap) {
    const obj = Object.create(null);
    for (const [k, v] of strMap) obj[k] = v;
    return obj;
}

// reverse complement; only A/T/G/C are mapped, every other char is kept (lib/kmers.js:31-38)
function complement(string) {
    let out = '';
    for (let i = string.length - 1; i >= 0; i -= 1) {
        const c = string[i];
        const m = complementMap.get(c);
        out += m === undefined ? c : m;
    }
    return out;
}

// legacy loop of the npm main (lib/index.js:60-73)
function kmers(line, kmerMap, length, preffix, step) {
    const stop = line.length - length + 1;
    let ini = 0;
    for (let index = 0; index < stop; index += 1) {
        const key = line.substring(ini, ini + length);
        if (key.startsWith(preffix)) kmerMap.set(key, (kmerMap.get(key) || 0) + 1);
        ini += step;
    }
    return true;
}

// Fold a packed native result into an existing, non-empty Map, preserving
// Map semantics: existing keys keep their position, new keys append in
// first-occurrence order.  (An empty Map is replaced by a KmerMap instead.)
function foldResult(map, res) {
    const keys = res.keys;
    const off = res.offsets;
    const cnt = res.counts;
    const n = cnt.length;
    const all = keys.latin1Slice(0, n ? off[n] : 0);
    for (let i = 0; i < n; i += 1) {
        const key = all.substring(off[i], off[i + 1]);
        const prev = map.get(key);
        map.set(key, prev === undefined ? cnt[i] : prev + cnt[i]);
    }
}

// GPUs of one count: this.devices (an array of HIP ordinals) or
// KMERHIP_DEVICES="0,1,..."; two or more shard the file over them (one
// result, merged over xGMI; kmer_params.ndev)
function devices(kmerObj) {
    if (Array.isArray(kmerObj.devices)) return kmerObj.devices;
    const env = process.env.KMERHIP_DEVICES;
    return env ? env.split(',').map(Number) : [];
}

const KMER_FLAG_UNORDERED = 16;
const KMER_FLAG_CANONICAL = 64;
function modeFlags(mode) {
    if (mode === undefined || mode === 'ordered') return 0;
    if (mode === 'unordered') return KMER_FLAG_UNORDERED;
    if (mode === 'canonical') return KMER_FLAG_CANONICAL;
    throw new Error(`kmerjs_amd: unknown mode '${mode}' (ordered, unordered, canonical)`);
}

function tooManyKeys(msg) {
    const e = new RangeError(msg);
    e.status = KMER_E_TOO_MANY_KEYS;
    return e;
}

class KmerJS {
    constructor(fastq = '', preffix = 'ATGAC', length = 16, step = 1,
        coverage = 1, progress = true, env = 'node') {
        this.fastq = fastq;
        this.preffix = preffix;
        this.kmerLength = length;
        this.step = step;
        this.progress = progress;
        this.coverage = coverage;
        this.evalue = new BN(0.05);
        this.kmerMap = new KmerMap('', [0], []);   // a Map (instanceof Map), filled in place by readFile()
        this.kmerMapSize = 0;
        this.env = env;
        this.maxKeys = MAP_MAX_KEYS;     // the reference Map's limit (lib/kmers.js:95)
        // extension: 'ordered' (the reference's Map, insertion order) or the
        // table modes for inputs whose Map is too large to build (BASELINE C3 /
        // C5): 'unordered' (the same keys and counts, sorted by key) and
        // 'canonical' (one key per {x, rc x} class; kmer_api.h KMER_FLAG_*)
        this.mode = 'ordered';
        this.batchBytes = 0;             // extension: input batch size (0 = the library's default)
        if (env === 'browser') this.fileDataRead = 0;
    }

    kmersInLine(line) {
        const k = this.kmerLength;
        const p = this.preffix;
        const stop = line.length - k;
        let ini = 0;
        for (let index = 0; index <= stop; index += 1) {
            const kmer = line.substring(ini, ini + k);
            if (kmer.startsWith(p)) this.kmerMap.set(kmer, (this.kmerMap.get(kmer) || 0) + 1);
            ini += this.step;
        }
    }

    readFile() {
        const kmerObj = this;
        // progress-stream is a Transform the file is piped through (lib/kmers.js:108-110, :139);
        // here the bytes never reach JS, so the stream carries only the events and ends
        const event = new stream.PassThrough();
        let lastProgress = null;
        event.progress = () => lastProgress;
        kmerObj.lines = 0;
        kmerObj.bytesRead = 0;
        kmerObj.linesPerChunk = 0;
        const promise = new Promise((resolve, reject) => {
            if (kmerObj.env !== 'node') {
                event.end();
                reject(new Error("kmerjs_amd: env '" + kmerObj.env + "' is not served by the GPU addon"));
                return;
            }
            let handle;
            try {
                // (the native result alone may not exceed the limit; a pre-filled
                // Map is checked again after the fold)
                handle = native().open(kmerObj.kmerLength, Buffer.from(String(kmerObj.preffix), 'latin1'),
                    kmerObj.step, Number(process.env.KMERHIP_DEVICE || 0), modeFlags(kmerObj.mode), kmerObj.maxKeys,
                    kmerObj.batchBytes || 0, devices(kmerObj));
            } catch (e) {
                event.end();
                reject(e);
                return;
            }
            // the progress-stream of lib/kmers.js:108-110: one 'progress' event
            // per input batch read (progress-stream's fields; bytesRead follows)
            const t0 = Date.now();
            let lastDone = 0, lastTotal = -1, finished = false;
            const emitProgress = (done, total) => {
                lastTotal = total;
                const runtime = (Date.now() - t0) / 1000;
                const speed = runtime > 0 ? done / runtime : 0;
                kmerObj.bytesRead = done;
                lastProgress = {
                    percentage: total ? (100 * done) / total : 0,
                    transferred: done,
                    length: total,
                    remaining: total > done ? total - done : 0,
                    eta: speed > 0 && total > done ? Math.round((total - done) / speed) : 0,
                    runtime: Math.round(runtime),
                    delta: done - lastDone,
                    speed,
                };
                event.emit('progress', lastProgress);
                lastDone = done;
            };
            // (batch events come from the reader thread; the completion may be
            // delivered before the last of them -- it then emits the final one
            // itself, and later arrivals are dropped, so events stay monotone and
            // end at the whole file before the promise resolves)
            const onProgress = (done, total) => {
                if (!finished) emitProgress(done, total);
            };
            native().countFile(handle, String(kmerObj.fastq), (err, res) => {
                native().close(handle);
                finished = true;
                if (err) {
                    event.end();
                    reject(err.status === KMER_E_TOO_MANY_KEYS ? tooManyKeys(err.message) : err);
                    return;
                }
                try {
                    if (kmerObj.kmerMap.size === 0 && kmerObj.kmerMap instanceof KmerMap) {
                        kmerObj.kmerMap.adopt(res, native().indexKeys);   // the same object, filled lazily (kmer_map.js)
                    } else {
                        // (a caller-supplied Map, empty or not: filled in place, then
                        // held to the reference Map's limit, lib/kmers.js:95)
                        foldResult(kmerObj.kmerMap, res);
                        if (kmerObj.kmerMap.size > kmerObj.maxKeys) throw tooManyKeys('Map maximum size exceeded');
                    }
                } catch (e) {
                    event.end();
                    reject(e);        // (never an exception escaping the completion callback)
                    return;
                }
                if (lastTotal < 0 || lastDone < lastTotal) {
                    let size = lastTotal;
                    if (size < 0) {
                        try { size = fs.statSync(String(kmerObj.fastq)).size; } catch (e) { size = lastDone; }
                    }
                    emitProgress(size, size);
                }
                kmerObj.lines = res.lines;
                if (kmerObj.progress) {
                    process.stdout.write(`Lines: ${res.lines} / Kmers: ${kmerObj.kmerMap.size}\r`);
                    process.stdout.write('\n                               \n');
                }
                kmerObj.kmerMapSize = kmerObj.kmerMap.size;
                event.end();
                resolve(kmerObj.kmerMap);
            }, onProgress);
        });
        return { promise, event };
    }
}

// README-style convenience (README.md:15): kmerjs(fastq, preffix, length, step) -> Promise<Map>
function kmerjs(fastq, preffix = 'ATGAC', length = 16, step = 1) {
    return new KmerJS(fastq, preffix, length, step, 1, false, 'node').readFile().promise;
}

module.exports = {
    complementMap, jsonToStrMap, complement, stringToMap, objectToMap, mapToJSON, KmerJS,
    kmers, kmerjs, KmerMap, version: () => native().version(), native, devices,
};
