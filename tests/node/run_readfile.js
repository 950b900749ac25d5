// readFile() on one file through the drop-in (tests/test_node.py): prints the
// sha256 of JSON.stringify([...map]), the Map size and kmerObj.lines.
'use strict';
const crypto = require('crypto');
const path = require('path');

const [file, prefix, k] = process.argv.slice(2);
const { KmerJS } = require(path.join(__dirname, '..', '..', 'kmerjs_amd', 'node', 'kmers.js'));
const kj = new KmerJS(file, prefix, Number(k), 1, 1, false, 'node');
kj.readFile().promise.then((map) => {
    const digest = crypto.createHash('sha256').update(JSON.stringify([...map]), 'utf8').digest('hex');
    process.stdout.write(JSON.stringify({ digest, size: map.size, lines: kj.lines }) + '\n');
}, (e) => {
    process.stdout.write(JSON.stringify({ error: String(e), status: e.status }) + '\n');
});
