/* kmerfinder.js — drop-in for kmerFinder's matching (lib/kmerFinderServer.js)
 * on the MI355X template matcher (include/kmer_match.h, via kmerhip.node).
 *
 * KmerFinderServer keeps the reference's constructor, findKmers(),
 * findMatches(kmerMap) and findFirstMatch(kmerMap):
 *   - 'winner' (lib/kmerFinderServer.js:736-849): firstMatch ->
 *     findKmersMatchesRedis (:171-226), findWinner (sort by uScore, first
 *     wins), matchSummary (:625-676), removeWinnerKmers (:778-789: the
 *     winner's k-mers are deleted from the caller's Map), getMatches
 *     (:791-830), until a winner is not significant or maxHits;
 *   - 'standard' (:857-874): every template with hits, in DB order
 *     (findMatchesMongoAggregation :452-522), summarised, sorted by score,
 *     rejected ones (undefined) last.
 * The joins and re-scoring run on the GPU; the statistics (lib/stats.js zScore,
 * fastp) are bignumber.js 2.x decimal arithmetic (package.json:61), restated
 * exactly with BigInt below.  lib/kmerFinderServer.js:7 sets BN.config({
 * ROUNDING_MODE: 2 }) on the one bignumber.js constructor lib/stats.js shares,
 * so dividedBy / sqrt round to 20 places with ROUND_CEIL and a bare round(dp)
 * is a ceiling; plus / minus / times are exact, round(dp, 6) is half-even.
 *
 * The template DB: the reference reads Redis (kmer -> [template JSON]) or
 * MongoDB (the ETL's documents, src/kmerPyToMongo.py:36-42), neither of which
 * is served here.  `url` names a JSON file instead: an array of the ETL's
 * documents {sequence, lengths, ulenght (or ulength / ulengths), species,
 * reads: [k-mer]} or {summary: {templates, totalLen, uniqueLens}, templates:
 * [...]}; loadTemplates(array, summary) does the same from memory.  A k-mer's
 * templates are in DB order.  Errors: the reference's 'No hits were found!...'
 * messages, as rejected promises.
 */
'use strict';
const fs = require('fs');
const drop = require('./kmers.js');

const { KmerJS, KmerMap } = drop;
const native = drop.native;

// ---------------------------------------------------------------------------
// decimals: n / 10^s with BigInt n (bignumber.js 2.x semantics)
// ---------------------------------------------------------------------------
const DP = 20;
const TEN = BigInt(10);
const pow10 = (e) => TEN ** BigInt(e);
const babs = (x) => (x < BigInt(0) ? -x : x);

class Dec {
    constructor(n, s) { this.n = n; this.s = s; }

    static of(x) {
        if (x instanceof Dec) return x;
        const t = String(x).toLowerCase();          // new BigNumber(number) reads its string form
        const [mant, ex = '0'] = t.split('e');
        const [ip, fp = ''] = mant.split('.');
        const n = BigInt(ip + fp);
        const s = fp.length - Number(ex);
        return s >= 0 ? new Dec(n, s) : new Dec(n * pow10(-s), 0);
    }

    _al(o) {
        o = Dec.of(o);
        const s = Math.max(this.s, o.s);
        return [this.n * pow10(s - this.s), o.n * pow10(s - o.s), s];
    }

    plus(o) { const [a, b, s] = this._al(o); return new Dec(a + b, s); }

    minus(o) { const [a, b, s] = this._al(o); return new Dec(a - b, s); }

    times(o) { o = Dec.of(o); return new Dec(this.n * o.n, this.s + o.s); }

    cmp(o) { const [a, b] = this._al(o); return a > b ? 1 : a < b ? -1 : 0; }

    // dividedBy: DP places, ROUND_CEIL (towards +Infinity)
    div(o) {
        o = Dec.of(o);
        const num = this.n * pow10(DP + o.s);
        const den = o.n * pow10(this.s);
        const neg = (num < BigInt(0)) !== (den < BigInt(0));
        const an = babs(num);
        const ad = babs(den);
        let q = an / ad;
        if (!neg && an % ad !== BigInt(0)) q += BigInt(1);
        return new Dec(neg ? -q : q, DP);
    }

    // sqrt: DP places, ROUND_CEIL (this >= 0)
    sqrt() {
        const e = 2 * DP - this.s;
        const num = e >= 0 ? this.n * pow10(e) : this.n;
        const den = e >= 0 ? BigInt(1) : pow10(-e);
        let t = isqrt(num / den);
        if (t * t * den !== num) t += BigInt(1);
        return new Dec(t, DP);
    }

    // mode 6: half-even; omitted: the configured ROUNDING_MODE, ROUND_CEIL
    round(dp, mode) {
        if (this.s <= dp) return this;
        const d = pow10(this.s - dp);
        const neg = this.n < BigInt(0);
        const a = babs(this.n);
        let q = a / d;
        const r = a % d;
        if (mode === 6) {
            const r2 = BigInt(2) * r;
            if (r2 > d || (r2 === d && q % BigInt(2) === BigInt(1))) q += BigInt(1);
        } else if (!neg && r !== BigInt(0)) {
            q += BigInt(1);
        }
        return new Dec(neg ? -q : q, dp);
    }

    toNumber() { return this.s === 0 ? Number(this.n) : Number(`${this.n}e-${this.s}`); }
}

function isqrt(n) {
    if (n < BigInt(2)) return n;
    let x = BigInt(Math.floor(Math.sqrt(Number(n))));      // start near the root, then Newton
    for (;;) {
        const y = (x + n / x) >> BigInt(1);
        if (y >= x) break;
        x = y;
    }
    while (x * x > n) x -= BigInt(1);
    while ((x + BigInt(1)) * (x + BigInt(1)) <= n) x += BigInt(1);
    return x;
}

const ETTA = new Dec(BigInt(1), 8);                 // lib/stats.js:6
const EVALUE = new Dec(BigInt(5), 2);               // lib/kmers.js:75
const FASTP = [
    ['10.7016', '1e-26'], ['10.4862', '1e-25'], ['10.2663', '1e-24'], ['10.0416', '1e-23'], ['9.81197', '1e-22'],
    ['9.5769', '1e-21'], ['9.33604', '1e-20'], ['9.08895', '1e-19'], ['8.83511', '1e-18'], ['8.57394', '1e-17'],
    ['8.30479', '1e-16'], ['8.02686', '1e-15'], ['7.73926', '1e-14'], ['7.4409', '1e-13'], ['7.13051', '1e-12'],
    ['6.8065', '1e-11'], ['6.46695', '1e-10'], ['6.10941', '1e-9'], ['5.73073', '1e-8'], ['5.32672', '1e-7'],
    ['4.89164', '1e-6'], ['4.41717', '1e-5'], ['3.89059', '1e-4'], ['3.29053', '1e-3'], ['2.57583', '0.01'],
    ['1.95996', '0.05'], ['1.64485', '0.1'],
].map(([a, b]) => [Dec.of(a), Dec.of(b)]);

// lib/stats.js:52-115
function fastp(z) {
    for (const [thr, p] of FASTP) if (z.cmp(thr) > 0) return p;
    return Dec.of(1);
}

// lib/stats.js:19-45
function zScore(r1, n1, r2, n2) {
    const p1 = Dec.of(r1).div(n1).plus(ETTA);
    const p2 = Dec.of(r2).div(n2).plus(ETTA);
    const p = Dec.of(r1).plus(r2).div(Dec.of(n1).plus(n2).plus(ETTA));
    const q = Dec.of(1).minus(p);
    const square = p.times(q).times(Dec.of(1).div(Dec.of(n1).plus(ETTA)).plus(Dec.of(1).div(Dec.of(n2).plus(ETTA))))
        .plus(ETTA).sqrt();
    return p1.minus(p2).div(square);
}

// matchSummary (lib/kmerFinderServer.js:625-676): a Map, or undefined
function matchSummary(querySize, sequence, match, first, hits, summary) {
    if (!(match.uScore > 0)) return undefined;
    const z = zScore(match.uScore, match.ulength, hits, summary.uniqueLens);
    const probability = fastp(z).times(summary.templates);
    if (EVALUE.cmp(probability) < 0) return undefined;
    const qs = Dec.of(querySize).plus(ETTA);
    const ul = Dec.of(match.ulength).plus(ETTA);
    const r2 = (x) => x.round(2, 6).toNumber();
    return new Map([
        ['template', sequence],
        ['score', match.uScore],
        ['expected', Dec.of(hits).times(match.ulength).div(summary.uniqueLens).round(0, 6).toNumber()],
        ['z', z.round(2).toNumber()],
        ['probability', probability.toNumber()],
        ['frac-q', r2(Dec.of(200 * match.uScore).div(qs))],
        ['frac-d', r2(Dec.of(100 * match.uScore).div(ul))],
        ['depth', r2(Dec.of(match.tScore).div(match.lengths))],
        ['kmers-template', match.ulength],
        ['total-frac-q', r2(Dec.of(200 * first.uScore).div(qs))],
        ['total-frac-d', r2(Dec.of(100 * first.uScore).div(ul))],
        ['total-temp-cover', r2(Dec.of(first.tScore).div(match.lengths))],
        ['species', match.species],
    ]);
}

// ---------------------------------------------------------------------------
// the template DB on the GPU
// ---------------------------------------------------------------------------
class TemplateDB {
    // templates: [{sequence, lengths, ulength, species, kmers | reads}]
    constructor(templates, summary, device = 0) {
        this.templates = templates.map((t) => ({
            sequence: t.sequence,
            lengths: t.lengths,
            ulength: t.ulength !== undefined ? t.ulength : t.ulenght !== undefined ? t.ulenght : t.ulengths,
            species: t.species,
        }));
        const lists = templates.map((t) => t.kmers || t.reads || []);
        let k = 0;
        for (const l of lists) if (l.length) { k = l[0].length; break; }
        const starts = new Float64Array(templates.length + 1);
        for (let i = 0; i < lists.length; i += 1) starts[i + 1] = starts[i] + lists[i].length;
        const keys = Buffer.from(lists.map((l) => l.join('')).join(''), 'latin1');
        if (keys.length !== starts[templates.length] * (k || 1)) {
            const e = new Error('kmerjs_amd: every template k-mer must have the same length');
            e.status = 2;
            throw e;
        }
        this.k = k || 1;
        this.handle = native().dbOpen(this.k, keys, starts, device);
        this.summary = summary || {
            templates: this.templates.length,
            totalLen: this.templates.reduce((a, t) => a + Number(t.lengths), 0),
            uniqueLens: this.templates.reduce((a, t) => a + Number(t.ulength), 0),
        };
    }

    static fromFile(file, device = 0) {
        const doc = JSON.parse(fs.readFileSync(file, 'utf8'));
        return Array.isArray(doc) ? new TemplateDB(doc, undefined, device)
            : new TemplateDB(doc.templates, doc.summary, device);
    }

    info() { return native().dbInfo(this.handle); }

    close() {
        if (this.handle) native().dbClose(this.handle);
        this.handle = null;
    }
}

// a Map's keys / counts in iteration order, packed for the matcher
function packQuery(kmerMap) {
    if (kmerMap instanceof KmerMap && kmerMap._packedOnly()) {
        return {
            n: kmerMap._n,
            keys: Buffer.from(kmerMap._all, 'latin1'),
            offsets: kmerMap._off instanceof Float64Array ? kmerMap._off : Float64Array.from(kmerMap._off),
            counts: kmerMap._cnt instanceof Float64Array ? kmerMap._cnt : Float64Array.from(kmerMap._cnt),
            keyAt: (i) => kmerMap._key(i),
            remove: (i) => kmerMap._deletePacked(i),
        };
    }
    const keys = [];
    const counts = [];
    for (const [k, v] of kmerMap) {
        keys.push(k);
        counts.push(Number(v));
    }
    const offsets = new Float64Array(keys.length + 1);
    // a key outside Latin-1 can never match: sent as '!' bytes
    const enc = keys.map((k) => (/[^\x00-\xff]/.test(k) ? '!'.repeat(k.length) : k));
    for (let i = 0; i < keys.length; i += 1) offsets[i + 1] = offsets[i] + enc[i].length;
    return {
        n: keys.length,
        keys: Buffer.from(enc.join(''), 'latin1'),
        offsets,
        counts: Float64Array.from(counts),
        keyAt: (i) => keys[i],
        remove: (i) => kmerMap.delete(keys[i]),
    };
}

function noHits(msg) { return new Error(msg); }

function templateEntry(kobj, db, m, q, t, u, ts) {
    const meta = db.templates[t];
    const entry = { tScore: ts, uScore: u, lengths: meta.lengths, ulength: meta.ulength, species: meta.species };
    let kmers = null;      // the k-mers Set, built on first use (lib/kmerFinderServer.js:198)
    Object.defineProperty(entry, 'kmers', {
        enumerable: true,
        get() {
            if (kmers === null) {
                kmers = new Set();
                for (const i of native().matchTemplateKmers(m, t)) kmers.add(q.keyAt(i));
            }
            return kmers;
        },
    });
    return entry;
}

// findKmersMatchesRedis: {templates: Map name -> entry (first-hit order), hits}
function firstRound(kobj, db, m, q) {
    const r = native().matchTemplates(m, 0);
    const templates = new Map();
    let hits = 0;
    for (let i = 0; i < r.tmpl.length; i += 1) {
        const t = r.tmpl[i];
        templates.set(db.templates[t].sequence, templateEntry(kobj, db, m, q, t, r.u[i], r.t[i]));
        hits += r.u[i];
    }
    return { templates, hits };
}

function progressLine(kobj, winner, header) {
    if (!kobj.progress) return;
    if (header) {
        process.stdout.write('Template\tScore\tExpected\tz\tp_value\tquery\tcoverage [%]\ttemplate coverage [%]\t'
            + 'depth\tKmers in Template\tDescription\n');
    }
    if (winner) {
        const g = (k) => winner.get(k);
        process.stdout.write(`${g('template')}\t${g('score')}\t${g('expected')}\t${g('z')}\t${g('probability')}\t`
            + `${g('frac-q')}\t${g('frac-d')}\t${g('depth')}\t${g('kmers-template')}\t${g('species')}\n`);
    }
}

function runWinner(kobj, kmerMap) {
    const db = kobj.templateDB();
    const q = packQuery(kmerMap);
    const m = native().matchOpen(db.handle, q.keys, q.offsets, q.counts);
    const results = [];
    let lastAlive = null;         // templates with hits at the last getMatches
    try {
        let w = native().matchWinner(m);
        if (w.hits === 0) throw noHits('No hits were found!');
        const first = firstRound(kobj, db, m, q);
        kobj.firstMatches = first.templates;
        for (;;) {
            const meta = db.templates[w.tmpl];
            const match = { uScore: w.uscore, tScore: w.tscore, lengths: meta.lengths, ulength: meta.ulength,
                species: meta.species };
            const winner = matchSummary(kobj.kmerMapSize, meta.sequence, match,
                { uScore: w.firstU, tScore: w.firstT }, w.hits, db.summary);
            if (results.length === 0) progressLine(kobj, null, true);
            if (!winner || EVALUE.cmp(winner.get('probability')) < 0) break;
            results.push(winner);
            progressLine(kobj, winner, false);
            native().matchRemove(m, w.tmpl);               // removeWinnerKmers + getMatches
            if (results.length >= kobj.maxHits) break;
            w = native().matchWinner(m);
            lastAlive = native().matchTemplates(m, 0).tmpl;
            if (w.hits === 0) throw noHits('No hits were found! (nHits === 0)');
        }
    } finally {
        // the reference deleted the winners' k-mers from the caller's Map, and
        // hit-less templates from firstMatches, as it went
        if (results.length) {
            const gone = native().matchRemoved(m, q.n);
            for (let i = 0; i < q.n; i += 1) if (gone[i]) q.remove(i);
            if (lastAlive !== null) {
                const alive = new Set(Array.from(lastAlive, (t) => db.templates[t].sequence));
                for (const name of [...kobj.firstMatches.keys()]) if (!alive.has(name)) kobj.firstMatches.delete(name);
            }
        }
        native().matchClose(m);
    }
    if (results.length === 0) throw noHits('No hits were found! (kmerResults.length === 0)');
    return results;
}

function runStandard(kobj, kmerMap) {
    const db = kobj.templateDB();
    const q = packQuery(kmerMap);
    const m = native().matchOpen(db.handle, q.keys, q.offsets, q.counts);
    try {
        const r = native().matchTemplates(m, 1);
        const templates = new Map();
        let hits = 0;
        for (let i = 0; i < r.tmpl.length; i += 1) {
            const t = r.tmpl[i];
            const meta = db.templates[t];
            templates.set(meta.sequence, { tScore: r.t[i], uScore: r.u[i], lengths: meta.lengths,
                ulength: meta.ulength, species: meta.species });
            hits += r.u[i];
        }
        if (hits === 0) throw noHits('No hits were found!');
        kobj.firstMatches = templates;
        const out = [];
        for (const [sequence, match] of templates) {
            out.push(matchSummary(kobj.kmerMapSize, sequence, match, match, hits, db.summary));
        }
        // sortKmerResults (:684-693) on a stable sort; undefined entries go last
        return out.sort((a, b) => b.get('score') - a.get('score'));
    } finally {
        native().matchClose(m);
    }
}

function later(fn) {
    return new Promise((resolve, reject) => setImmediate(() => {
        try {
            resolve(fn());
        } catch (e) {
            reject(e);
        }
    }));
}

class KmerFinderServer extends KmerJS {
    constructor(fastq, preffix = 'ATGAC', length = 16, step = 1, coverage = 1,
        progress = true, db = 'mongo', url = 'mongodb://localhost:27017/Kmers', collection = 'genomes',
        method = 'standard', maxHits = 100) {
        super(fastq, preffix, length, step, coverage, progress, 'node');
        this.url = url;
        this.dbType = db;
        this.method = method;
        this.collection = collection;
        this.firstMatches = new Map();
        this.maxHits = maxHits;
        this._db = null;
    }

    // the GPU template DB: loadTemplates(), or the JSON file named by url
    templateDB() {
        if (this._db === null) {
            if (typeof this.url !== 'string' || !fs.existsSync(this.url)) {
                throw new Error(`kmerjs_amd: no template DB (url '${this.url}' is not a JSON file; `
                    + 'Redis / MongoDB are not served)');
            }
            this._db = TemplateDB.fromFile(this.url, Number(process.env.KMERHIP_DEVICE || 0));
        }
        return this._db;
    }

    loadTemplates(templates, summary) {
        if (this._db) this._db.close();
        this._db = new TemplateDB(templates, summary, Number(process.env.KMERHIP_DEVICE || 0));
        return this;
    }

    findKmers() { return this.readFile().promise; }

    findMatches(kmerMap) {
        if (this.method === 'standard') return later(() => runStandard(this, kmerMap));
        if (this.method === 'winner') return later(() => runWinner(this, kmerMap));
        throw new Error('Scoring scheme unknown');
    }

    findFirstMatch(kmerMap) {
        if (this.method === 'standard') return later(() => runStandard(this, kmerMap));
        if (this.method === 'winner') {
            return later(() => {
                const db = this.templateDB();
                const q = packQuery(kmerMap);
                const m = native().matchOpen(db.handle, q.keys, q.offsets, q.counts);
                const r = firstRound(this, db, m, q);
                if (r.hits === 0) {
                    native().matchClose(m);
                    throw noHits('No hits were found!');
                }
                return r;       // (the match stays open for the lazy kmers Sets; freed with it)
            });
        }
        throw new Error('Scoring scheme unknown');
    }

    findMatchesTest(kmerMap) { return later(() => runWinner(this, kmerMap)); }

    close() {
        if (this._db) this._db.close();
        this._db = null;
    }
}

module.exports = { KmerFinderServer, TemplateDB, Dec, zScore, fastp, matchSummary };
