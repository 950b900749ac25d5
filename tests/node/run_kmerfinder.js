// Drives kmerjs_amd/node/kmerfinder.js for tests/test_node.py.
//   node run_kmerfinder.js stats SPEC.json  -> matchSummary / zScore of each case (CPU only)
//   node run_kmerfinder.js match SPEC.json  -> findMatches of each case on the GPU
// SPEC (match): {cases: [{templates, summary, method, maxHits,
//                          query: [[key, count], ...] | file: {path, prefix, k}}]}
// Output: one JSON line; per case {results | error, remaining: [[key, count], ...]}.
'use strict';
const fs = require('fs');
const path = require('path');

const repo = path.resolve(__dirname, '..', '..');
const kf = require(path.join(repo, 'kmerjs_amd', 'node', 'kmerfinder.js'));

const [mode, specFile] = process.argv.slice(2);
const spec = JSON.parse(fs.readFileSync(specFile, 'utf8'));

function asPairs(r) { return r === undefined ? null : [...r]; }

async function main() {
    const out = [];
    if (mode === 'stats') {
        for (const c of spec.cases) {
            const match = { uScore: c.u, tScore: c.ts, lengths: c.lengths, ulength: c.ulength, species: 's' };
            const r = kf.matchSummary(c.qsize, 'NC_1', match, { uScore: c.fu, tScore: c.ft }, c.hits, c.summary);
            out.push(asPairs(r));
        }
    } else {
        for (const c of spec.cases) {
            const kobj = new kf.KmerFinderServer(c.file ? c.file.path : '', c.file ? c.file.prefix : 'ATGAC',
                c.file ? c.file.k : 16, 1, 1, false, 'file', '', 'genomes', c.method, c.maxHits || 100);
            kobj.loadTemplates(c.templates, c.summary);
            let map;
            if (c.file) {
                map = await kobj.findKmers();          // a KmerMap (lazy), kmerMapSize set by readFile
            } else {
                map = new Map(c.query);
                kobj.kmerMapSize = map.size;
            }
            const rec = {};
            try {
                rec.results = (await kobj.findMatches(map)).map(asPairs);
            } catch (e) {
                rec.error = e.message;
            }
            rec.remaining = [...map];
            rec.firstMatches = [...kobj.firstMatches.keys()];
            kobj.close();
            out.push(rec);
        }
    }
    process.stdout.write(JSON.stringify(out) + '\n');
}

main().catch((e) => {
    process.stdout.write(JSON.stringify({ fatal: String(e.stack || e) }) + '\n');
    process.exit(1);
});
