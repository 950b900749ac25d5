// Node-side tests of the drop-in module, written like the reference's own
// test/kmers.js (KATs :12-52).  Mode "cpu": no GPU calls.  Mode "gpu":
// readFile() parity against the golden vectors (ordered Map, counts, lines).
'use strict';
const assert = require('assert');
const crypto = require('crypto');
const fs = require('fs');
const path = require('path');

const mode = process.argv[2] || 'cpu';
const repo = path.resolve(__dirname, '..', '..');
const lib = require(path.join(repo, 'kmerjs_amd', 'node', 'kmers.js'));
const { KmerJS, complement } = lib;
const results = [];
function check(name, fn) {
    try { fn(); results.push({ name, ok: true }); } catch (e) { results.push({ name, ok: false, err: String(e.stack || e) }); }
}

function cpuTests() {
    check('exports match lib/kmers.js', () => {
        for (const n of ['complementMap', 'jsonToStrMap', 'complement', 'stringToMap', 'objectToMap', 'mapToJSON', 'KmerJS']) {
            assert.ok(n in lib, n);
        }
    });
    check('ATGACGCAATACTCCT in kmersInLine()', () => {     // test/kmers.js:12-19
        const kmers = new KmerJS();
        const seq = `NTTTATGACGCAATACTCCTCTCTCCTTCGTGGTCTTGCAGCGGGTTCTGC
                   ATTTTTATTCCTTTTTGCCCCAACGGCATTCGCGGCGGAACAAACCGTTG`;
        kmers.kmersInLine(seq);
        assert.strictEqual([...kmers.kmerMap][0][0], 'ATGACGCAATACTCCT');
    });
    check('complement(ATGACCTGAGAGCCTT) = AAGGCTCTCAGGTCAT', () => {   // test/kmers.js:21-26
        assert.strictEqual(complement('ATGACCTGAGAGCCTT'), 'AAGGCTCTCAGGTCAT');
        assert.strictEqual(complement('acgtNX\r'), '\rXNtgca');
    });
    check('map helpers', () => {
        const m = lib.stringToMap('{"b":2,"a":1}');
        assert.deepStrictEqual([...m], [['b', 2], ['a', 1]]);
        const o = lib.mapToJSON(m);
        assert.strictEqual(o.b, 2);
        assert.deepStrictEqual([...lib.jsonToStrMap({ x: 3 })], [['x', 3]]);
        assert.deepStrictEqual([...lib.objectToMap({ y: 4 })], [['y', 4]]);
    });
    check('defaults and evalue', () => {
        const k = new KmerJS('f.fastq');
        assert.strictEqual(k.preffix, 'ATGAC');
        assert.strictEqual(k.kmerLength, 16);
        assert.strictEqual(k.step, 1);
        assert.strictEqual(k.evalue.cmp(0.05), 0);
        assert.ok(k.kmerMap instanceof Map);
    });
    check('legacy kmers()', () => {
        const m = new Map();
        lib.kmers('ACGTACGT', m, 4, '', 2);
        assert.deepStrictEqual([...m], [['ACGT', 2], ['GTAC', 1], ['GT', 1], ['', 1]]);
    });
    check('addon loads', () => {
        assert.ok(/gfx950/.test(lib.version()));
    });
}

function sha(s) { return crypto.createHash('sha256').update(s, 'utf8').digest('hex'); }

async function gpuTests() {
    const golden = JSON.parse(fs.readFileSync(path.join(repo, 'tests', 'golden', 'golden.json'), 'utf8'));
    const want = golden.cases.filter((c) => c.step === 1 && [16, 21, 31].includes(c.k)
        && ['ATGAC', ''].includes(c.prefix));
    for (const c of want) {
        const file = path.join(repo, 'tests', 'golden', 'inputs', c.input);
        const kj = new KmerJS(file, c.prefix, c.k, c.step, 1, false, 'node');
        const { promise, event } = kj.readFile();
        let progressed = false;
        event.on('progress', () => { progressed = true; });
        try {
            const map = await promise;
            const ok = sha(JSON.stringify([...map])) === c.digest && kj.lines === c.lines
                && kj.kmerMapSize === c.size && progressed && map === kj.kmerMap;
            results.push({ name: `readFile ${c.input} '${c.prefix}' k=${c.k}`, ok,
                err: ok ? undefined : `size ${map.size} vs ${c.size}, lines ${kj.lines} vs ${c.lines}` });
        } catch (e) {
            results.push({ name: `readFile ${c.input} '${c.prefix}' k=${c.k}`, ok: false, err: String(e) });
        }
    }
    // reference test/kmers.js:28-35 and :45-52 (via .promise: the reference tests call .then on the handle)
    const short = await new KmerJS(path.join(repo, 'tests', 'golden', 'inputs', 'test_short.fastq'), 'ATGAC', 16, 1, 1, false).readFile().promise;
    results.push({ name: 'readFile(test_short.fastq) should have 2 kmer', ok: short.size === 2 });
    const long = await new KmerJS(path.join(repo, 'tests', 'golden', 'inputs', 'test_long.kmer.fastq'), 'ATGAC', 16, 1, 1, false).readFile().promise;
    results.push({ name: 'readFile(test_long.kmer.fastq) should have 401 kmers', ok: long.size === 401 });
    // a missing file rejects (reference: uncaught stream error)
    try {
        await new KmerJS('/nonexistent.fastq').readFile().promise;
        results.push({ name: 'missing file rejects', ok: false });
    } catch (e) {
        results.push({ name: 'missing file rejects', ok: e.status === 1 });
    }
    // the Map is a real mutable Map, consumers may add / delete keys
    short.set('db', 'Kmers'); short.delete('ATGACGCAATACTCCT');
    results.push({ name: 'result Map is mutable', ok: short.size === 2 && short.get('db') === 'Kmers' });
}

(async () => {
    if (mode === 'cpu') cpuTests(); else await gpuTests();
    process.stdout.write(JSON.stringify(results) + '\n');
})();
