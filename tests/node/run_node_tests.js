// Node-side tests of the drop-in module, written like the reference's own
// test/kmers.js (KATs :12-52).  Mode "cpu": no GPU calls.  Mode "gpu":
// readFile() parity against the golden vectors (ordered Map, counts, lines).
'use strict';
const assert = require('assert');
const crypto = require('crypto');
const fs = require('fs');
const path = require('path');
const stream = require('stream');

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
    check('constructor Map is the Map readFile() fills; event is a Readable', () => {
        const k = new KmerJS('f.fastq', 'ATGAC', 16, 1, 1, false, 'browser');
        assert.ok(k.kmerMap instanceof Map && k.kmerMap instanceof lib.KmerMap && k.kmerMap.size === 0);
        const rf = k.readFile();                     // (browser env: rejects without touching the GPU)
        assert.ok(rf.event instanceof stream.Readable && typeof rf.event.pipe === 'function');
        assert.strictEqual(rf.event.progress(), null);
        rf.promise.catch(() => {});
    });
    check('legacy kmers()', () => {
        const m = new Map();
        lib.kmers('ACGTACGT', m, 4, '', 2);
        assert.deepStrictEqual([...m], [['ACGT', 2], ['GTAC', 1], ['GT', 1], ['', 1]]);
    });
    check('addon loads', () => {
        assert.ok(/gfx950/.test(lib.version()));
    });
    check('KmerMap follows Map semantics (random operations vs a real Map)', () => {
        // packed result of n distinct keys, as the addon hands it over
        const n = 500;
        const keys = [];
        for (let i = 0; i < n; i += 1) keys.push('K' + ((i * 7919) % 100003).toString(36) + 'x'.repeat(i % 5));
        const buf = Buffer.from(keys.join(''), 'latin1');
        const off = new Float64Array(n + 1);
        for (let i = 0; i < n; i += 1) off[i + 1] = off[i] + keys[i].length;
        const cnt = new Float64Array(n);
        for (let i = 0; i < n; i += 1) cnt[i] = (i % 13) + 1;
        const km = lib.KmerMap.fromNative({ keys: buf, offsets: off, counts: cnt });
        const ref = new Map();
        for (let i = 0; i < n; i += 1) ref.set(keys[i], cnt[i]);
        assert.ok(km instanceof Map);
        const same = () => {
            assert.strictEqual(km.size, ref.size);
            assert.deepStrictEqual([...km], [...ref]);
            assert.deepStrictEqual([...km.keys()], [...ref.keys()]);
            assert.deepStrictEqual([...km.values()], [...ref.values()]);
            const a = []; km.forEach((v, k, m) => { assert.strictEqual(m, km); a.push([k, v]); });
            assert.deepStrictEqual(a, [...ref]);
        };
        same();                                     // before any keyed access (lazy)
        let x = 1;
        const rnd = (m) => { x = (x * 1103515245 + 12345) % 2147483648; return x % m; };
        for (let step = 0; step < 3000; step += 1) {
            const op = rnd(6);
            const key = rnd(3) === 0 ? 'new' + rnd(40) : keys[rnd(n)];
            if (op === 0) { km.set(key, step); ref.set(key, step); }
            else if (op === 1) assert.strictEqual(km.delete(key), ref.delete(key));
            else if (op === 2) assert.strictEqual(km.get(key), ref.get(key));
            else if (op === 3) assert.strictEqual(km.has(key), ref.has(key));
            else if (op === 4) { km.set('db', 'Kmers'); ref.set('db', 'Kmers'); }
            else { km.delete('db'); ref.delete('db'); }
            if (step % 500 === 0) same();
        }
        same();
        assert.strictEqual(lib.mapToJSON(km)[keys[1]], ref.get(keys[1]));
        km.clear(); ref.clear();
        same();
    });
    check('KmerMap hash index at scale, delete by packed index', () => {
        const n = 50000;
        const keys = [];
        for (let i = 0; i < n; i += 1) keys.push('ATGAC' + ((i * 2654435761) >>> 0).toString(4).padStart(11, 'A'));
        const uniq = [...new Set(keys)];
        const buf = Buffer.from(uniq.join(''), 'latin1');
        const off = new Float64Array(uniq.length + 1);
        for (let i = 0; i < uniq.length; i += 1) off[i + 1] = off[i] + uniq[i].length;
        const cnt = new Float64Array(uniq.length).map((_, i) => i + 1);
        const km = lib.KmerMap.fromNative({ keys: buf, offsets: off, counts: cnt });
        assert.ok(km._packedOnly());
        for (let i = 0; i < uniq.length; i += 97) assert.strictEqual(km.get(uniq[i]), i + 1);
        assert.strictEqual(km.get('ATGACZZZZZZZZZZZ'), undefined);
        assert.strictEqual(km.has(uniq[5].slice(0, 15)), false);
        assert.strictEqual(km.has(42), false);
        assert.ok(km._deletePacked(7) && !km._deletePacked(7));
        assert.strictEqual(km.has(uniq[7]), false);
        assert.strictEqual(km.size, uniq.length - 1);
        assert.ok(!km._packedOnly());
        assert.strictEqual([...km.keys()][7], uniq[8]);
    });
    check('native KmerMap index (indexKeys) = the JS table; same Map semantics', () => {
        const n = 20000;
        const keys = [];
        for (let i = 0; i < n; i += 1) keys.push('AC' + ((i * 40503 + 7) >>> 0).toString(4).padStart(9, 'G') + '\xe9\r'.slice(0, i % 3));
        const uniq = [...new Set(keys)];
        const buf = Buffer.from(uniq.join(''), 'latin1');
        const off = new Float64Array(uniq.length + 1);
        for (let i = 0; i < uniq.length; i += 1) off[i + 1] = off[i] + uniq[i].length;
        const cnt = new Float64Array(uniq.length).map((_, i) => i + 1);
        const res = { keys: buf, offsets: off, counts: cnt };
        const js = lib.KmerMap.fromNative(res);
        const nat = lib.KmerMap.fromNative(res, lib.native().indexKeys);
        assert.deepStrictEqual(nat._index(), js._index());
        for (let i = 0; i < uniq.length; i += 37) assert.strictEqual(nat.get(uniq[i]), i + 1);
        assert.strictEqual(nat.get('ACZ'), undefined);
        nat.set(uniq[3], 0); nat.delete(uniq[4]); nat.set('new', 1);
        assert.deepStrictEqual([...nat].slice(2, 5), [[uniq[2], 3], [uniq[3], 0], [uniq[5], 6]]);
        assert.deepStrictEqual([...nat].pop(), ['new', 1]);
        assert.throws(() => lib.native().indexKeys(buf, off, uniq.length, 3), RangeError);
    });
    check('legacy npm main (lib/index.js) exports and fields', () => {
        const legacy = require(path.join(repo, 'kmerjs_amd', 'node', 'index.js'));
        for (const name of ['kmers', 'complement', 'KmerJSClient', 'KmerJSServer']) assert.ok(name in legacy, name);
        const s = new legacy.KmerJSServer('x.fastq');
        assert.strictEqual(s.preffix, 'ATGAC');
        assert.strictEqual(s.length, 16);
        assert.strictEqual(s.step, 1);
        assert.strictEqual(s.uKmers, 0);
        assert.deepStrictEqual(s.db, { type: 'mongo', url: 'mongodb://localhost:27017/Kmers' });
        assert.strictEqual(s.evalue.cmp(0.05), 0);
        assert.strictEqual(s.mapToJSON(new Map([['a', 1]])), '{"a":1}');
        const c = new legacy.KmerJSClient('x.fastq', 'AT', 5, 1, 1, '', 'json');
        assert.strictEqual(c.url, 'http://localhost:3000/kmers');
        assert.strictEqual(c.db.url, '../test_data/db.json');
        assert.strictEqual(legacy.complement('ATGACCTGAGAGCCTT'), 'AAGGCTCTCAGGTCAT');
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
    // the resolved Map is the constructor's Map object (lib/kmers.js:76, :178), and
    // event is a Readable that ends after the count, like progress-stream (:108, :183)
    {
        const file = path.join(repo, 'tests', 'golden', 'inputs', 'test_long.kmer.fastq');
        const kj = new KmerJS(file, 'ATGAC', 16, 1, 1, false);
        const before = kj.kmerMap;
        const { promise, event } = kj.readFile();
        let ended = false;
        event.on('end', () => { ended = true; });
        event.resume();
        const m = await promise;
        await new Promise((r) => setImmediate(r));
        const last = event.progress();
        const ok = m === before && kj.kmerMap === before && m.size === 401 && event instanceof stream.Readable
            && ended && last !== null && last.transferred === fs.statSync(file).size;
        results.push({ name: 'readFile fills the constructor Map; event is a Readable that ends', ok,
            err: ok ? undefined : `same ${m === before} size ${m.size} ended ${ended} last ${JSON.stringify(last)}` });
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
    results.push({ name: 'result Map is mutable', ok: short.size === 2 && short.get('db') === 'Kmers'
        && short instanceof Map && [...short][1][0] === 'db' });
    // more distinct keys than the Map may hold: the promise rejects with a
    // RangeError (the reference's Map.set throws, lib/kmers.js:95)
    {
        const kj = new KmerJS(path.join(repo, 'tests', 'golden', 'inputs', 'test_long.kmer.fastq'), 'ATGAC', 16, 1, 1, false);
        kj.maxKeys = 100;
        try {
            await kj.readFile().promise;
            results.push({ name: 'too many keys rejects', ok: false });
        } catch (e) {
            results.push({ name: 'too many keys rejects', ok: e instanceof RangeError && e.status === 5 });
        }
        // a pre-filled Map: the fold checks the limit after merging
        const kp = new KmerJS(path.join(repo, 'tests', 'golden', 'inputs', 'test_long.kmer.fastq'), 'ATGAC', 16, 1, 1, false);
        kp.maxKeys = 401;
        kp.kmerMap.set('pre', 1);
        try {
            await kp.readFile().promise;
            results.push({ name: 'pre-filled Map over the limit rejects', ok: false });
        } catch (e) {
            results.push({ name: 'pre-filled Map over the limit rejects', ok: e instanceof RangeError });
        }
        const kq = new KmerJS(path.join(repo, 'tests', 'golden', 'inputs', 'test_long.kmer.fastq'), 'ATGAC', 16, 1, 1, false);
        kq.kmerMap.set('pre', 1);
        const mq = await kq.readFile().promise;
        results.push({ name: 'pre-filled Map folds', ok: mq.size === 402 && [...mq][0][0] === 'pre' && mq === kq.kmerMap });
    }
    // legacy npm main: KmerJSServer/KmerJSClient.findKmers (lib/index.js:250-306, :402-408, :327-332)
    {
        const legacy = require(path.join(repo, 'kmerjs_amd', 'node', 'index.js'));
        const cases = golden.cases.filter((c) => c.step === 1 && [16, 31].includes(c.k) && ['ATGAC', ''].includes(c.prefix));
        for (const c of cases) {
            const file = path.join(repo, 'tests', 'golden', 'inputs', c.input);
            for (const Cls of [legacy.KmerJSServer, legacy.KmerJSClient]) {
                const o = new Cls(file, c.prefix, c.k, c.step);
                try {
                    const m = await o.findKmers();
                    const ok = sha(JSON.stringify([...m])) === c.digest && m.size === c.size && o.uKmers === 0;
                    results.push({ name: `${Cls.name}.findKmers ${c.input} '${c.prefix}' k=${c.k}`, ok });
                } catch (e) {
                    results.push({ name: `${Cls.name}.findKmers ${c.input}`, ok: false, err: String(e) });
                }
            }
        }
    }
    // multi-GPU through readFile(): two shards on a device group (ordinal 0 twice
    // on a one-GPU box), merged into the same ordered Map
    for (const c of golden.cases.filter((x) => x.step === 1 && x.k === 16 && ['ATGAC', ''].includes(x.prefix))) {
        const kj = new KmerJS(path.join(repo, 'tests', 'golden', 'inputs', c.input), c.prefix, c.k, 1, 1, false);
        kj.devices = [0, 0];
        try {
            const m = await kj.readFile().promise;
            const ok = sha(JSON.stringify([...m])) === c.digest && kj.lines === c.lines;
            results.push({ name: `readFile on devices [0,0] ${c.input} '${c.prefix}'`, ok });
        } catch (e) {
            results.push({ name: `readFile on devices [0,0] ${c.input}`, ok: false, err: String(e) });
        }
    }
    // readFile() progress (lib/kmers.js:108-110): one 'progress' event per input
    // batch, with real byte counts; bytesRead follows; same Map as one batch
    {
        const file = path.join(repo, 'tests', 'golden', 'inputs', 'test_long.kmer.fastq');
        const size = fs.statSync(file).size;
        const c = golden.cases.find((x) => x.input === 'test_long.kmer.fastq' && x.prefix === 'ATGAC' && x.k === 16
            && x.step === 1);
        for (const devs of [[], [0, 0, 0]]) {
            const kj = new KmerJS(file, 'ATGAC', 16, 1, 1, false);
            kj.batchBytes = 1 << 16;
            kj.devices = devs;
            const ev = [];
            const rf = kj.readFile();
            rf.event.on('progress', (p) => ev.push(p));
            try {
                const m = await rf.promise;
                await new Promise((r) => setImmediate(r));      // (events queued before the result)
                const last = ev[ev.length - 1] || {};
                const mono = ev.every((p, i) => i === 0 || p.transferred >= ev[i - 1].transferred);
                const ok = sha(JSON.stringify([...m])) === c.digest && ev.length >= 2 && mono
                    && last.transferred === size && last.length === size && last.percentage === 100
                    && kj.bytesRead === size;
                results.push({ name: `readFile progress events [${devs}] (${ev.length})`, ok });
            } catch (e) {
                results.push({ name: `readFile progress events [${devs}]`, ok: false, err: String(e) });
            }
        }
    }
    // table modes through readFile() (BASELINE C3 / C5 from the reference's entry
    // point): the same keys and counts as the ordered Map, sorted by key; and
    // canonical classes; on one device and on a device group
    {
        const file = path.join(repo, 'tests', 'golden', 'inputs', 'test_long.kmer.fastq');
        const kj = new KmerJS(file, '', 21, 1, 1, false);
        const ordered = await kj.readFile().promise;
        const want = [...ordered].sort((a, b) => (a[0] < b[0] ? -1 : a[0] > b[0] ? 1 : 0));
        for (const devs of [[], [0, 0]]) {
            const ku = new KmerJS(file, '', 21, 1, 1, false);
            ku.mode = 'unordered';
            ku.devices = devs;
            const kc = new KmerJS(file, '', 21, 1, 1, false);
            kc.mode = 'canonical';
            kc.devices = devs;
            try {
                const mu = await ku.readFile().promise;
                const mc = await kc.readFile().promise;
                const okU = JSON.stringify([...mu]) === JSON.stringify(want);
                const okC = mc.size > 0 && [...mc].every(([k, v]) => k <= complement(k)
                    && ordered.get(k) === (k === complement(k) ? 2 * v : v));
                results.push({ name: `readFile table modes [${devs}]`, ok: okU && okC, detail: { okU, okC } });
            } catch (e) {
                results.push({ name: `readFile table modes [${devs}]`, ok: false, err: String(e) });
            }
        }
    }
    // close() while a count is in flight: closed when it completes (no use after free)
    {
        const nat = lib.native();
        const h = nat.open(16, Buffer.from('ATGAC', 'latin1'), 1, 0);
        const done = new Promise((resolve) => {
            nat.countFile(h, path.join(repo, 'tests', 'golden', 'inputs', 'test_long.kmer.fastq'), (err, res) => {
                resolve(!err && res.counts.length === 401);
            });
        });
        nat.close(h);
        let reuse = false;
        try { nat.countFile(h, 'x', () => {}); } catch (e) { reuse = true; }
        results.push({ name: 'close while busy is deferred', ok: (await done) && reuse });
    }
}

(async () => {
    if (mode === 'cpu') cpuTests(); else await gpuTests();
    process.stdout.write(JSON.stringify(results) + '\n');
})();
