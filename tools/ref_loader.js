// Loads the UNMODIFIED reference hot path (/root/reference/lib/kmers.js) under
// node 12 for golden-vector generation. Container-only tool: it reads the
// reference at run time and is never shipped, imported by product code, or run
// on the GPU box (SURVEY.md Appendix B recipe; nothing of the reference is
// copied into this repository).
//
// The reference is ES2015-module syntax normally run through babel
// (.babelrc:1-4). We rewrite its six `import X from 'y'` lines into requires of
// stand-ins for the four absent npm deps (none of which touch the data path:
// SURVEY.md §8c), strip `export`, and compile it as a CommonJS module.
'use strict';
const fs = require('fs');
const path = require('path');
const Module = require('module');
const stream = require('stream');

const REF = process.env.KMERJS_REF || '/root/reference/lib/kmers.js';

function stubRequire(name) {
    switch (name) {
    case 'bignumber.js': return function BN(v) { this.v = v; };
    case 'bluebird': return Promise;
    case 'console': return console;
    case 'stream': return stream;
    case 'progress-stream': return () => new stream.PassThrough();
    case 'filereader-stream': return () => { throw new Error('browser only'); };
    default: return require(name);
    }
}

function loadReference() {
    let src = fs.readFileSync(REF, 'utf8');
    src = src.replace(/^import (\w+) from '([^']+)';$/mg, 'const $1 = __req(\'$2\');');
    src = src.replace(/^export (let|function|class) /mg, '$1 ');
    src = 'const __req = module.__stubRequire;\n' + src +
        '\nmodule.exports = {complementMap, jsonToStrMap, complement, stringToMap,' +
        ' objectToMap, mapToJSON, KmerJS};\n';
    const m = new Module(REF, null);
    m.filename = REF;
    m.paths = Module._nodeModulePaths(path.dirname(REF));
    m.__stubRequire = stubRequire;
    m._compile(src, REF);
    return m.exports;
}

module.exports = { loadReference };

// CLI: node ref_loader.js <fastq> <prefix> <k> <step> [out.json]
// Prints (or writes) JSON.stringify([...map]) of the reference readFile() result.
function runBatch() {
    const ref = loadReference();
    const cases = JSON.parse(fs.readFileSync(0, 'utf8'));
    let idx = 0;
    const next = () => {
        if (idx >= cases.length) return;
        const c = cases[idx++];
        const kj = new ref.KmerJS(c.file, c.prefix, c.k, c.step, 1, false, 'node');
        kj.readFile().promise.then((map) => {
            process.stdout.write(JSON.stringify({ id: c.id, lines: kj.lines, kmerMapSize: kj.kmerMapSize,
                entries: JSON.stringify([...map]) }) + '\n');
            next();
        });
    };
    next();
}

// --time <fastq> <prefix> <k> <progress 0|1>: wall time of the unmodified
// readFile() (promise resolved), the Map's size and ordered digest (sha256 of
// JSON.stringify([...map]), first 16 hex), as one JSON line on stderr (with
// progress=1 the reference writes a line to stdout per input line).
function runTime() {
    const [file, prefix, k, prog] = process.argv.slice(3);
    const ref = loadReference();
    const kj = new ref.KmerJS(file, prefix, parseInt(k, 10), 1, 1, prog === '1', 'node');
    const t0 = process.hrtime.bigint();
    kj.readFile().promise.then((map) => {
        const t1 = process.hrtime.bigint();
        const digest = require('crypto').createHash('sha256').update(JSON.stringify([...map]), 'utf8')
            .digest('hex').slice(0, 16);
        process.stderr.write(JSON.stringify({ seconds: Number(t1 - t0) / 1e9, size: map.size, lines: kj.lines,
            sum: [...map.values()].reduce((a, b) => a + b, 0), digest, progress: prog === '1' }) + '\n');
    });
}

if (require.main === module && process.argv[2] === '--batch') {
    runBatch();
} else if (require.main === module && process.argv[2] === '--time') {
    runTime();
} else if (require.main === module) {
    const [file, prefix, k, step, out] = process.argv.slice(2);
    const ref = loadReference();
    const kj = new ref.KmerJS(file, prefix, parseInt(k, 10), parseInt(step, 10), 1, false, 'node');
    const t0 = process.hrtime.bigint();
    kj.readFile().promise.then((map) => {
        const t1 = process.hrtime.bigint();
        const s = JSON.stringify([...map]);
        const meta = { seconds: Number(t1 - t0) / 1e9, size: map.size, lines: kj.lines };
        if (out) {
            fs.writeFileSync(out, s);
            process.stdout.write(JSON.stringify(meta) + '\n');
        } else {
            process.stdout.write(s + '\n');
        }
    });
}

